"""All-reduce bandwidth of the framework's data plane (SURVEY §7.1 bench/allreduce_bw).

Sweeps message sizes through ``Tree(...).comm.all_reduce`` -- the native RCCL
communicator on GPUs (``csrc/comm/communicator.h``), the gloo process-group
communicator on CPU -- and, on GPUs, the same sizes through torch's own
``dist.all_reduce`` on an NCCL(=RCCL) group for comparison.  Prints one JSON
line per (path, size): time per call (max over ranks), algorithm bandwidth
``bytes / t`` and bus bandwidth ``algbw * 2 (n-1) / n`` (the per-link figure a
ring over xGMI is bound by).

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
        scripts/allreduce_bw.py [--device cpu] [--min-kb 64] [--max-mb 256]

The reference has no such benchmark (no published bandwidth);
its cost claim is T*log2(N) for the tree all-reduce (lua/AllReduceEA.md:26-30).
With one rank the collective is issued through RCCL anyway
(DISTLEARN_RCCL_WORLD1=1) so the launch/graph overhead is measured.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"])
    ap.add_argument("--dtype", default="float32", choices=["float32", "bfloat16"])
    ap.add_argument("--min-kb", type=float, default=64)
    ap.add_argument("--max-mb", type=float, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--torch", type=int, default=1, help="also time torch.distributed's NCCL group (GPU only)")
    a = ap.parse_args(argv)
    os.environ.setdefault("DISTLEARN_RCCL_WORLD1", "1")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")

    import torch
    import torch.distributed as dist

    from torch_distlearn_amd import Tree

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.device == "cuda":
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        sync = torch.cuda.synchronize
    else:
        dev = torch.device("cpu")
        sync = lambda: None  # noqa: E731
    dt = getattr(torch, a.dtype)
    tree = Tree(rank + 1, world, host=os.environ["MASTER_ADDR"], port=int(os.environ["MASTER_PORT"]), device=dev)
    comm = tree.comm

    paths = [("distlearn", lambda t: comm.all_reduce(t))]
    if a.device == "cuda" and a.torch and world > 1:
        grp = dist.new_group(list(range(world)), backend="nccl")
        paths.append(("torch.distributed", lambda t: dist.all_reduce(t, group=grp)))

    esz = torch.empty((), dtype=dt).element_size()
    sizes = []
    b = int(a.min_kb * 1024)
    while b <= int(a.max_mb * (1 << 20)):
        sizes.append(b)
        b *= 4
    buf = torch.zeros(sizes[-1] // esz, dtype=dt, device=dev)
    rows = []
    for name, fn in paths:
        for nbytes in sizes:
            t = buf[: nbytes // esz]
            for _ in range(a.warmup):
                fn(t)
            sync()
            comm.barrier()
            sync()
            t0 = time.perf_counter()
            for _ in range(a.iters):
                fn(t)
            sync()
            el = torch.tensor([(time.perf_counter() - t0) / a.iters], dtype=torch.float64)
            comm.all_reduce_host(el, "max")
            sec = float(el)
            algbw = nbytes / sec / 1e9
            row = {"path": name, "bytes": nbytes, "n_ranks": world, "dtype": a.dtype, "device": a.device,
                   "us": round(sec * 1e6, 2), "algbw_GBps": round(algbw, 2),
                   "busbw_GBps": round(algbw * 2 * (world - 1) / world, 2) if world > 1 else None}
            rows.append(row)
            if rank == 0:
                print(json.dumps(row), flush=True)
    # zeros in, zeros out on every rank (a corrupted transfer would show here)
    assert int(torch.count_nonzero(buf)) == 0, "all-reduce of zeros returned non-zero data"
    comm.barrier()
    return rows


if __name__ == "__main__":
    main()
