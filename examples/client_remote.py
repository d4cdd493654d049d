#!/usr/bin/env python3
"""Multi-host Tree built by hand (reference: examples/client_remote.lua:31-41,
client_remote.sh).  Every node passes the root's ``--host/--port`` and its own
``--nodeIndex``; ``--base`` is the reference's tree arity (accepted; the
collectives are RCCL rings/trees over xGMI/RoCE, gloo on CPU).

The reference script mixes a CPU node and a GPU node in ONE tree
(client_remote.sh:4-6).  ``--backend gloo`` reproduces that (gloo reduces CPU
and GPU tensors); the default ``auto`` uses RCCL when ``--cuda`` is given.
The reference file itself is stale (it calls AsyncEA with the AllReduceEA
signature); this one trains the CIFAR convnet with AllReduceEA as
the reference intended.

    # node 1 (root)                      # node 2
    python examples/client_remote.py --nodeIndex 1 --numNodes 2 --host 10.0.0.1 --port 8080
    python examples/client_remote.py --nodeIndex 2 --numNodes 2 --host 10.0.0.1 --port 8080 --cuda
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torch_distlearn_amd import AllReduceEA, FlatParams, Tree  # noqa: E402
from torch_distlearn_amd.data import Dataset  # noqa: E402
from torch_distlearn_amd.launch import add_node_flags, device_of, node_opts  # noqa: E402
from torch_distlearn_amd.models import CifarConvNet  # noqa: E402
from torch_distlearn_amd.ops.flat import flat_sgd_  # noqa: E402


def main():
    ap = add_node_flags(argparse.ArgumentParser(description=__doc__.split("\n\n")[0]), batch=32, lr=0.01)
    ap.add_argument("--backend", default="auto", choices=["auto", "rccl", "nccl", "gloo"])
    ap.add_argument("--epochs", type=int, default=1)
    ap.add_argument("--maxSteps", type=int, default=0)
    ap.add_argument("--trainSize", type=int, default=50000)
    ap.add_argument("--tau", type=int, default=10)
    ap.add_argument("--alpha", type=float, default=0.2)
    opt = ap.parse_args()
    node_opts(opt)
    dev = device_of(opt)
    tree = Tree(opt.nodeIndex, opt.numNodes, opt.base, None, None, opt.host, opt.port, device=dev,
                backend=opt.backend)
    per_node = math.ceil(opt.batchSize / opt.numNodes)  # client_remote.lua:56-57
    ds = Dataset("cifar10", opt.nodeIndex, opt.numNodes, synthetic_size=opt.trainSize, device=dev)
    cd = torch.bfloat16 if dev.type == "cuda" else torch.float32
    b = ds.sampledBatcher("permutation", per_node, dtype=cd, seed=opt.nodeIndex)
    model = CifarConvNet(seed=0).to(dev)
    flat = FlatParams(model, grads=True)
    ea = AllReduceEA(tree, opt.tau, opt.alpha)
    ea.synchronizeParameters(flat)
    for epoch in range(opt.epochs):
        nb = b.numBatches() if not opt.maxSteps else min(opt.maxSteps, b.numBatches())
        for _ in range(nb):
            x, y = b.getBatch()
            flat.grad.zero_()
            loss = model.loss(model(x, compute_dtype=cd), y)
            loss.backward()
            flat_sgd_(flat, opt.learningRate)
            ea.averageParameters(flat)
        ea.synchronizeCenter(flat)
        if opt.nodeIndex == 1:
            print(f"epoch {epoch + 1}: loss {float(loss.detach()):.4f}")
    tree.comm.barrier()


if __name__ == "__main__":
    main()
