#!/usr/bin/env python3
"""Headline benchmark: whole-node images/sec of the reference's CIFAR-10
convnet trained with AllReduceSGD (BASELINE.json "metric"), bf16 compute,
synthetic CIFAR-shaped data, random-init weights.

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

With ``--gpus N > 1`` and no torch.distributed environment (WORLD_SIZE
unset), bench.py launches itself: the parent spawns N child processes (one
rank per GPU: RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free
MASTER_PORT), never touches the GPU and never execs, forwards rank 0's JSON
line as its own last stdout line, and exits non-zero (killing the siblings) as
soon as any child fails or the launch times out -- the reference's launchers
fork their own N processes the same way (examples/cifar10-cuda.sh:4-7).

One rank per GPU; gradients are all-reduced over RCCL (xGMI) in buckets that
overlap backward; the timed region is EXACTLY K full training steps (forward,
backward, gradient all-reduce, 1/n normalisation, SGD update) bracketed by a
barrier + device synchronisation on both sides; the reported time is the MAX
over ranks.  Weak scaling: the per-GPU batch is fixed (default 128 = the
reference's per-client AsyncEA batch, examples/AsyncEASGD.sh:36-40), the global
batch is N x per-GPU batch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_VALUE = None  # the reference publishes no numbers


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (weak scaling; cifar10 128, resnet50 256)")
    ap.add_argument("--backend", default=os.environ.get("DISTLEARN_BENCH_BACKEND", "hip"), choices=["hip", "torch"])
    ap.add_argument("--algo", default="sgd", choices=["sgd", "ea", "async"],
                    help="sgd = AllReduceSGD (headline), ea = AllReduceEA (tau, alpha), "
                         "async = AsyncEA: rank 0 parameter server + N-1 clients (BASELINE configs 2-4)")
    ap.add_argument("--model", default="cifar10", choices=["cifar10", "resnet50"],
                    help="resnet50 = BASELINE config 5 (ImageNet shape 224x224; stride-1 1x1 and 3x3 convs on the "
                         "HIP MFMA kernels, HIP BatchNorm; see models/resnet.py for the rest)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu = gloo plumbing check of the same code path (tests only; not a benchmark)")
    ap.add_argument("--tau", type=int, default=10)
    ap.add_argument("--alpha", type=float, default=0.2)
    ap.add_argument("--graph", type=int, default=1,
                    help="capture the step in a hipGraph (default 1).  ResNet-50: one step from the same state "
                         "differs between graph and eager by 2.0e-3 (relative, all gradients) while two eager runs "
                         "differ by 2.4e-3 and eager vs fp32 by 3.5e-2 (scripts/diag_r50_graph.py, "
                         "profiles/r2_resnet50_graph_diag.txt): the round-1 loss drift after 45 steps was bf16 "
                         "run-to-run noise amplified by a memorising synthetic run, not a graph bug")
    ap.add_argument("--bucket-mb", type=float, default=None,
                    help="gradient all-reduce bucket size (default: cifar10 1 MiB = 3 buckets "
                         "{conv4+bn4+fc, conv3+bn3, conv1..bn2}; resnet50 16 MiB)")
    ap.add_argument("--lr", type=float, default=None,
                    help="SGD learning rate (default: cifar10 0.1 = examples/cifar10.lua:7; resnet50 0.02)")
    ap.add_argument("--overlap", type=int, default=1, help="bucketed all-reduce overlapped with backward")
    ap.add_argument("--grad-comm-dtype", default=os.environ.get("DISTLEARN_GRAD_COMM_DTYPE", "fp32"),
                    choices=["fp32", "bf16"],
                    help="gradient all-reduce wire dtype (bf16: half the xGMI bytes, count in an fp32 side slot); "
                         "with --algo async: the AsyncEA delta push")
    ap.add_argument("--nworld-path", type=int, default=0,
                    help="1 = run the MULTI-NODE step configuration on one GPU (diagnostic, not the headline): the "
                         "bucket all-reduces go through RCCL at world 1 (DISTLEARN_RCCL_WORLD1=1), so the trainer "
                         "materialises every gradient for them (no one-node slab deferral / side SGD), the executor "
                         "takes its overlap policy (every candidate timed and reported unless DISTLEARN_POLICY "
                         "forces one)")
    ap.add_argument("--hold-cus", type=int, default=0,
                    help="with --nworld-path: hold R CUs during the timed region with workgroups of RCCL's "
                         "all-reduce footprint (csrc/testing/diag.hip occupy_cus; the worst case of a collective "
                         "overlapping the whole step); the time is then taken with GPU events")
    ap.add_argument("--launch-timeout", type=float, default=1800.0,
                    help="self-launch (--gpus N > 1 without torch.distributed.run): seconds before the children "
                         "are killed and bench.py exits non-zero")
    return ap.parse_args()


def _self_launch(a) -> int:
    """Spawn ``a.gpus`` ranks of this script as child processes (no exec, no
    GPU use in this parent), forward rank 0's JSON line, fail fast."""
    import signal
    import socket
    import subprocess
    import threading

    n = a.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs, lines, readers = [], [], []
    sys.stdout.flush()

    def pump(r, stream):
        for raw in iter(stream.readline, ""):
            if r == 0 and raw.startswith("{") and '"metric"' in raw:
                lines.append(raw.rstrip("\n"))
            else:  # everything else (RCCL banners, other ranks) goes to stderr
                sys.stderr.write(raw if r == 0 else f"[rank {r}] {raw}")
        stream.close()

    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DISTLEARN_SELF_LAUNCHED="1")
        p = subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                             stdout=subprocess.PIPE, text=True, start_new_session=True)
        procs.append(p)
        t = threading.Thread(target=pump, args=(r, p.stdout), daemon=True)
        t.start()
        readers.append(t)

    def kill_all():
        for p in procs:
            if p.poll() is None:
                try:
                    os.killpg(p.pid, signal.SIGKILL)
                except OSError:
                    pass
        for p in procs:
            p.wait()

    def on_term(signum, frame):
        kill_all()
        sys.exit(128 + signum)

    signal.signal(signal.SIGTERM, on_term)
    deadline = time.time() + a.launch_timeout
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
            if bad:
                r, rc = bad[0]
                print(f"bench.py: rank {r} exited with code {rc}; stopping the other ranks", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            if time.time() > deadline:
                print(f"bench.py: ranks still running after --launch-timeout {a.launch_timeout:.0f} s; killing them",
                      file=sys.stderr)
                rc = 124
                break
            time.sleep(0.05)
    finally:
        kill_all()
        for t in readers:
            t.join(timeout=5)
    if rc == 0:
        if not lines:
            print("bench.py: rank 0 printed no result line", file=sys.stderr)
            return 1
        print(lines[-1], flush=True)
    return rc


METRICS = {
    ("cifar10", "sgd"): "images/sec (whole node) CIFAR-10 AllReduceSGD",
    ("cifar10", "ea"): "images/sec (whole node) CIFAR-10 AllReduceEA",
    ("cifar10", "async"): "images/sec (whole node, clients) CIFAR-10 AsyncEA",
    ("resnet50", "sgd"): "images/sec (whole node) ResNet-50 AllReduceSGD",
    ("resnet50", "ea"): "images/sec (whole node) ResNet-50 AllReduceEA",
    ("resnet50", "async"): "images/sec (whole node, clients) ResNet-50 AsyncEA",
}
MODEL_DESC = {
    "cifar10": "cifar10-convnet (examples/cifar10.lua, 4.33M params)",
    "resnet50": "resnet50 (ImageNet shape 224x224, 25.6M params)",
}


def main():
    a = parse()
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(_self_launch(a))  # before torch is imported: the parent never touches the GPU
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if a.algo == "async" and world < 2:
        print("bench.py: --algo async needs >= 2 ranks (1 server + clients)", file=sys.stderr)
        sys.exit(2)
    cpu = a.device == "cpu"
    if a.nworld_path:
        if world != 1 or cpu:
            print("bench.py: --nworld-path rehearses the multi-node step on ONE GPU", file=sys.stderr)
            sys.exit(2)
        os.environ["DISTLEARN_RCCL_WORLD1"] = "1"
        os.environ.setdefault("DISTLEARN_POLICY_SELECT", "1")
    if cpu:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
    else:
        ndev = torch.cuda.device_count()  # does not initialise the GPU
        if ndev < world and os.environ.get("DISTLEARN_ALLOW_SHARED_GPU", "0") != "1":
            # one rank per GPU (RCCL refuses two ranks on one GPU): fail fast
            print(f"bench.py: --gpus {world} needs {world} GPUs, this node has {ndev}", file=sys.stderr)
            sys.exit(2)
        if local >= ndev:
            # DISTLEARN_ALLOW_SHARED_GPU=1: more ranks than GPUs (a functional
            # rehearsal of the multi-rank path on a small box; not a benchmark)
            print(f"bench.py: rank {rank}: LOCAL_RANK {local} >= {ndev} GPUs, sharing GPU {local % ndev}",
                  file=sys.stderr)
            local = local % ndev
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")
    batch = a.batch or (128 if a.model == "cifar10" else 256)
    if a.lr is None:
        a.lr = 0.1 if a.model == "cifar10" else 0.02
    if a.bucket_mb is None:
        a.bucket_mb = 1.0 if a.model == "cifar10" else 16.0
    backend = a.backend if (a.model == "cifar10" and not cpu) else "torch"
    if backend == "torch" and not cpu and os.environ.get("DISTLEARN_MIOPEN_FIND", "1") == "1":
        # MIOpen solver search per conv shape: only matters for the MIOpen A/B modes
        # (every ResNet-50 conv is on the HIP kernels by default); runs in the warm-up
        # steps, before the timed region (r2: 32.69 vs 33.93 ms/step, profiles/r2_bench_resnet50.txt)
        torch.backends.cudnn.benchmark = True
    cdt = torch.float32 if cpu else torch.bfloat16

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet, ResNet50
    from torch_distlearn_amd.utils.color_print import set_verbose

    set_verbose(False)  # one JSON line on stdout

    tree = Tree(rank + 1, world, host=os.environ["MASTER_ADDR"], port=int(os.environ["MASTER_PORT"]), device=dev)
    model = (CifarConvNet(seed=0) if a.model == "cifar10" else ResNet50(seed=0)).to(dev)
    is_server = a.algo == "async" and rank == 0
    # the workers that train: all ranks, or the AsyncEA clients (ranks 1..N-1)
    workers = list(range(1, world)) if a.algo == "async" else list(range(world))
    wgroup = dist.new_group(workers, backend="gloo") if a.algo == "async" else None

    def worker_barrier():
        if wgroup is None:
            tree.comm.barrier()
        else:
            dist.barrier(group=wgroup)

    dt, loss, comm = 0.0, None, {}
    if is_server:
        from torch_distlearn_amd import AsyncEA, FlatParams

        flat = FlatParams(model, grads=False, shadow_bf16=not cpu)
        server = AsyncEA(tree, None, None, None, None, None, world - 1, 0, a.tau, a.alpha,
                         delta_wire=a.grad_comm_dtype)
        server.initServer(flat)
        while server.syncServer(flat):
            pass
    else:
        tr = DataParallelTrainer(model, tree, lr=a.lr, algo=a.algo, tau=a.tau, alpha=a.alpha, backend=backend,
                                 compute_dtype=cdt, bucket_bytes=int(a.bucket_mb * (1 << 20)), overlap=bool(a.overlap),
                                 graph=bool(a.graph) and not cpu, max_batch=batch,
                                 grad_comm_dtype=a.grad_comm_dtype if a.algo in ("sgd", "async") else "fp32")
        tr.synchronize_parameters()
        if a.model == "cifar10":
            # synthetic CIFAR-10-shaped uint8 dataset resident in HBM (this rank's
            # partition of 50k images); the batch of every step is selected by a
            # device-side permutation sampler and gathered + normalised + padded
            # inside the (graph-captured) step -- the real data path, not a
            # pre-made tensor
            from torch_distlearn_amd.data import DeviceLoader, PartitionedDataset

            n_local = max(batch, 50000 // len(workers))
            g = torch.Generator(device=dev).manual_seed(1234 + rank)
            imgs = torch.randint(0, 256, (n_local, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
            labs = torch.randint(0, 10, (n_local,), device=dev, generator=g)
            loader = DeviceLoader(PartitionedDataset(imgs, labs, device=dev), "permutation", batch, seed=rank)
            step_args = None
        else:
            g = torch.Generator(device=dev).manual_seed(1234 + rank)
            nb = 2
            xs = torch.randn(nb, batch, 224, 224, 3, device=dev, generator=g).to(cdt)
            ys = torch.randint(0, 1000, (nb, batch), device=dev, generator=g)
            step_args = lambda i: (xs[i % nb], ys[i % nb])  # noqa: E731
        # steps per replayed graph: a timed window of at most 32 steps is ONE replay of a graph
        # holding exactly those steps (the driver's 20: 0.3307 vs 0.3335 ms/step as 16 + 4,
        # = the 600-step figure 0.3305, profiles/r3_unroll_ab.txt); longer runs replay 32-step
        # graphs (16 measured 1.3 % faster than 8, profiles/r2_unroll20_ab.txt; 32 vs 16:
        # 0.2994 / 0.3008 / 0.3007 vs 0.3012 / 0.3035 / 0.3010 ms, profiles/r4_prep_next_ab.txt)
        unroll = int(os.environ.get("DISTLEARN_UNROLL", str(a.steps if 1 < a.steps <= 32 else 32)))
        if step_args is None:  # device loader: unrolled graph replays of complete steps
            tr.run(loader, a.warmup, unroll=unroll)
        else:
            for i in range(a.warmup):
                wl = tr.step(*step_args(i))
                if os.environ.get("DISTLEARN_BENCH_TRACE", "") == "sync":
                    print(f"warmup {i} loss {float(wl):.4f} |p| {float(tr.flat.data.norm()):.4e} "
                          f"|g| {float(tr.flat.grad.norm()):.4e}", file=sys.stderr, flush=True)
        if step_args is None:
            tr.prepare(loader, unroll)  # (run() already did; explicit: no capture may fall in the timed region)
        comm = {}
        if (len(workers) > 1 or a.nworld_path) and a.algo == "sgd" and not cpu:
            # communication profile: HIP events around every bucket all-reduce, read from
            # replays of a captured one-step graph (the timed schedule; eager steps when
            # the model has no device loader), OUTSIDE the timed region; training state
            # is restored after
            comm = tr.comm_profile(loader if step_args is None else step_args, steps=6, replay=True)
        captures0 = tr.captures
        hold = None
        if a.hold_cus > 0 and not cpu:
            from torch_distlearn_amd import _native

            hold_stream = torch.cuda.Stream(device=dev)
            sink = torch.zeros(4096, device=dev)
            # outlasts the timed steps (<= 2 s); the window is timed with events on the step stream
            _native.testing().occupy_cus(a.hold_cus, min(2_000_000, a.steps * 1500 + 50_000), sink.data_ptr(),
                                         hold_stream.cuda_stream)
            torch.cuda._sleep(2_000_000)  # the holding workgroups land first
            hold = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
        else:
            sync()
        worker_barrier()
        if hold is None:
            sync()
        else:
            hold[0].record()
        probe = os.environ.get("DISTLEARN_BENCH_PROBE", "") == "1" and not cpu  # debug: where the window goes
        if probe:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        if probe:
            ev0.record()
        if step_args is None:
            loss = tr.run(loader, a.steps, unroll=unroll)
        else:
            trace = os.environ.get("DISTLEARN_BENCH_TRACE", "")  # debug: per-step losses (stderr)
            hist = []
            for i in range(a.steps):
                loss = tr.step(*step_args(i))
                if trace == "sync":
                    print(f"step {i} loss {float(loss):.4f}", file=sys.stderr, flush=True)
                elif trace:
                    hist.append(loss.detach().clone())
            for i, l in enumerate(hist):
                print(f"step {i} loss {float(l):.4f}", file=sys.stderr, flush=True)
        if probe:
            ev1.record()
            t_sub = time.perf_counter() - t0
        if hold is not None:
            hold[1].record()
        sync()
        if probe:
            t_sync = time.perf_counter() - t0
        worker_barrier()
        sync()
        dt = time.perf_counter() - t0
        if hold is not None:
            dt = hold[0].elapsed_time(hold[1]) / 1e3  # the holding kernel outlives the window
        if probe:
            print(f"probe: window {dt * 1e3:.3f} ms, host enqueue {t_sub * 1e3:.3f} ms, first sync {t_sync * 1e3:.3f} ms, "
                  f"GPU events {ev0.elapsed_time(ev1):.3f} ms", file=sys.stderr, flush=True)
        if tr.captures != captures0:
            raise RuntimeError(f"bench.py: {tr.captures - captures0} hipGraph capture(s) inside the timed region")
        tr.finish()
    # max over ranks (the AsyncEA server contributes 0); loss from the first worker
    t = torch.tensor([dt, float(loss.float().item()) if (loss is not None and rank == workers[0]) else -1e30],
                     dtype=torch.float64)
    tree.comm.all_reduce_host(t, "max")
    dt, lval = float(t[0]), float(t[1])
    # which device each rank ran on (a SCALE record must show N distinct GPUs)
    devs = torch.full((world,), -1, dtype=torch.int64)
    devs[rank] = -1 if cpu else torch.cuda.current_device()
    tree.comm.all_reduce_host(devs, "max")
    ex = getattr(tr, "executor", None) if not is_server else None
    policy = {
        "rccl_world": getattr(tree.comm, "world_size", world) if type(tree.comm).__name__ == "RcclCommunicator"
        else 0,
        "comm": type(tree.comm).__name__,
        "device_ids": sorted(set(int(d) for d in devs.tolist())),
        "nccl_max_nchannels": os.environ.get("NCCL_MAX_NCHANNELS"),
        # RCCL channel cap (maxCTAs) of the gradient communicator: measured with the
        # overlap policy at world > 1 (engine.py select_policy), 0 = no collective runs
        "channel_cap": getattr(tree.comm, "channel_cap", None),
        "cu_reserve": getattr(ex, "cu_reserve", None),
        "dgrad_stages": getattr(ex, "dgrad_stages", None),
        # the wire dtype actually used (world 1: no collective, fp32)
        "grad_comm_dtype": getattr(tr, "grad_comm_dtype", "fp32") if not is_server else "fp32",
        "delta_wire": a.grad_comm_dtype if a.algo == "async" else None,
        # world > 1: the overlap policy measured on this machine during warm-up
        # (engine.py select_policy: every candidate's ms per step, max over ranks)
        "policy": getattr(tr, "policy", None) if not is_server else None,
    }
    if a.nworld_path:
        policy["nworld_path"] = {
            "what": "multi-node step configuration on one GPU: bucket all-reduces through RCCL at world 1, "
                    "gradients materialised for them",
            "fused_slab_reduce": getattr(tr, "_fused_reduce", None), "held_cus": a.hold_cus}
    ms = dt / a.steps * 1e3
    imgs = batch * len(workers) * a.steps / dt
    if rank == 0:
        out = {
            "metric": METRICS[(a.model, a.algo)],
            "value": round(imgs, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else round(imgs / BASELINE_VALUE, 4),
            "dtype": "fp32" if cpu else "bf16",
            "data": ("synthetic CIFAR-10-shaped uint8 dataset in HBM (50k images split over the workers), "
                     "device-side permutation sampler, gather+normalise inside the step; random-init weights")
            if a.model == "cifar10" else "synthetic ImageNet-shaped bf16 batches, random-init weights",
            "config": {"model": MODEL_DESC[a.model],
                       "global_batch": batch * len(workers), "per_gpu_batch": batch, "seq_len": None,
                       "parallelism": f"dp{len(workers)}" + ("+ps1" if a.algo == "async" else ""), "algo": a.algo,
                       "backend": (backend if a.model == "cifar10" or cpu
                                   else "torch autograd over the hand-written HIP conv/BN/head kernels"),
                       "hipgraph": bool(a.graph), "bucket_mb": a.bucket_mb, **policy,
                       **({"tau": a.tau, "alpha": a.alpha} if a.algo != "sgd" else {})},
            "final_loss": round(lval, 4),
        }
        if comm:
            out["comm"] = {**comm, "method": f"rank 0, {comm.get('source', 'eager steps')}, "
                                             "6 calibration steps outside the timed region"}
        print(json.dumps(out), flush=True)
    tree.comm.barrier()


if __name__ == "__main__":
    main()
