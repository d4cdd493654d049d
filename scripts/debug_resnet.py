"""Per-step losses of ResNet-50 training on one GPU (eager vs hipGraph, lr sweep)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import Tree
from torch_distlearn_amd.engine import DataParallelTrainer
from torch_distlearn_amd.models import ResNet50

ap = argparse.ArgumentParser()
ap.add_argument("--graph", type=int, default=0)
ap.add_argument("--lr", type=float, default=0.1)
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=12)
ap.add_argument("--port", type=int, default=29701)
ap.add_argument("--bucket-mb", type=float, default=4.0)
ap.add_argument("--sync", type=int, default=1, help="0: no host sync between steps (losses cloned on the stream)")
ap.add_argument("--sync-params", type=int, default=0, help="call synchronize_parameters() first (as bench.py)")
ap.add_argument("--seed", type=int, default=0)
a = ap.parse_args()
dev = torch.device("cuda", 0)
tree = Tree(1, 1, host="127.0.0.1", port=a.port, device=dev)
m = ResNet50(seed=0).to(dev)
tr = DataParallelTrainer(m, tree, lr=a.lr, backend="torch", compute_dtype=torch.bfloat16, graph=bool(a.graph),
                         bucket_bytes=int(a.bucket_mb * (1 << 20)))
if a.sync_params:
    tr.synchronize_parameters()
g = torch.Generator(device=dev).manual_seed(a.seed)
x = torch.randn(2, a.batch, 224, 224, 3, device=dev, generator=g).to(torch.bfloat16)
y = torch.randint(0, 1000, (2, a.batch), device=dev, generator=g)
hist = []
for i in range(a.steps):
    loss = tr.step(x[i % 2], y[i % 2])
    if a.sync:
        gn = float(tr.flat.grad[64:].norm())
        print(f"graph={a.graph} lr={a.lr} step {i}: loss {float(loss):.4f} |g| {gn:.3e} "
              f"|p| {float(tr.flat.data.norm()):.3e}", flush=True)
    else:
        hist.append((loss.detach().clone(), tr.flat.data.norm(), tr.flat.grad[64:].norm()))
for i, (l, p, gn) in enumerate(hist):
    print(f"graph={a.graph} nosync step {i}: loss {float(l):.4f} |g| {float(gn):.3e} |p| {float(p):.3e}", flush=True)
