#!/usr/bin/env python3
"""Headline benchmark: whole-node images/sec of the reference's CIFAR-10
convnet trained with AllReduceSGD (BASELINE.json "metric"), bf16 compute,
synthetic CIFAR-shaped data, random-init weights.

    python bench.py --gpus N --steps K --warmup W           (N == 1)
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

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
    ap.add_argument("--batch", type=int, default=128, help="per-GPU batch (weak scaling)")
    ap.add_argument("--backend", default=os.environ.get("DISTLEARN_BENCH_BACKEND", "hip"), choices=["hip", "torch"])
    ap.add_argument("--algo", default="sgd", choices=["sgd", "ea"])
    ap.add_argument("--graph", type=int, default=1, help="capture the step in a hipGraph")
    ap.add_argument("--bucket-mb", type=float, default=4.0)
    ap.add_argument("--lr", type=float, default=0.1)
    return ap.parse_args()


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print(f"bench.py: --gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes", file=sys.stderr)
            sys.exit(2)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29517")

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet

    tree = Tree(rank + 1, world, host=os.environ["MASTER_ADDR"], port=int(os.environ["MASTER_PORT"]), device=dev)
    model = CifarConvNet(seed=0).to(dev)
    graph = bool(a.graph) and a.algo == "sgd"
    tr = DataParallelTrainer(model, tree, lr=a.lr, algo=a.algo, backend=a.backend, compute_dtype=torch.bfloat16,
                             bucket_bytes=int(a.bucket_mb * (1 << 20)), graph=graph, max_batch=a.batch)
    tr.synchronize_parameters()

    # synthetic CIFAR-shaped data: NHWC bf16, normalised; labels uniform over 10 classes
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    nb = 8
    xs = torch.randn(nb, a.batch, 32, 32, 3, device=dev, generator=g).to(torch.bfloat16)
    ys = torch.randint(0, 10, (nb, a.batch), device=dev, generator=g)

    for i in range(a.warmup):
        tr.step(xs[i % nb], ys[i % nb])
    torch.cuda.synchronize()
    tree.comm.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(a.steps):
        loss = tr.step(xs[i % nb], ys[i % nb])
    torch.cuda.synchronize()
    tree.comm.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64)
    tree.comm.all_reduce_host(t, "max")
    dt = float(t.item())
    ms = dt / a.steps * 1e3
    imgs = a.batch * world * a.steps / dt
    lval = float(loss.float().item())
    if rank == 0:
        out = {
            "metric": "images/sec (whole node) CIFAR-10 AllReduceSGD" if a.algo == "sgd"
            else "images/sec (whole node) CIFAR-10 AllReduceEA",
            "value": round(imgs, 1),
            "unit": "images/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None if BASELINE_VALUE is None else round(imgs / BASELINE_VALUE, 4),
            "dtype": "bf16",
            "data": "synthetic (CIFAR-10 shaped 32x32x3, random-init weights)",
            "config": {"model": "cifar10-convnet (examples/cifar10.lua, 4.33M params)",
                       "global_batch": a.batch * world, "per_gpu_batch": a.batch, "seq_len": None,
                       "parallelism": f"dp{world}", "algo": a.algo, "backend": a.backend, "hipgraph": graph,
                       "bucket_mb": a.bucket_mb},
            "final_loss": round(lval, 4),
        }
        print(json.dumps(out), flush=True)
    tree.comm.barrier()


if __name__ == "__main__":
    main()
