#!/usr/bin/env python3
"""MNIST convnet steps/s on one MI355X at the reference's per-node batch of 1
(examples/mnist.lua:33): the fused one-kernel HIP step vs the PyTorch-ops
path, both hipGraph-captured (and torch eager), AllReduceSGD engine, lr 0.01.
Prints one JSON line per configuration."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--only", default=None, help="e.g. hip-graph / torch-graph (profiling)")
    a = ap.parse_args()
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import MnistConvNet

    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29593, device=dev)
    g = torch.Generator(device=dev).manual_seed(0)
    xs = torch.randn(64, a.batch, 1024, device=dev, generator=g)
    ys = torch.randint(0, 10, (64, a.batch), device=dev, generator=g)
    for backend, graph in (("hip", True), ("hip", False), ("torch", True), ("torch", False)):
        if a.only and a.only != f"{backend}-{'graph' if graph else 'eager'}":
            continue
        m = MnistConvNet(seed=0).to(dev)
        tr = DataParallelTrainer(m, tree, lr=0.01, backend=backend, compute_dtype=torch.float32, graph=graph,
                                 max_batch=a.batch)
        tr.synchronize_parameters()
        for i in range(20):
            tr.step(xs[i % 64], ys[i % 64])
        torch.cuda.synchronize()
        n = a.steps if graph or backend == "hip" else a.steps // 4
        t0 = time.perf_counter()
        for i in range(n):
            loss = tr.step(xs[i % 64], ys[i % 64])
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"model": "mnist-convnet (examples/mnist.lua)", "batch": a.batch, "backend": backend,
                          "hipgraph": graph, "steps": n, "us_per_step": round(dt / n * 1e6, 2),
                          "steps_per_s": round(n / dt, 1), "final_loss": round(float(loss), 4)}), flush=True)


if __name__ == "__main__":
    main()
