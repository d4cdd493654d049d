#!/usr/bin/env python3
"""CIFAR-10 convnet trained with AllReduceSGD (reference: examples/cifar10.lua).

Same flags as the reference (``--nodeIndex --numNodes --batchSize
--learningRate --cuda --gpu``); ``--batchSize`` is the GLOBAL batch split
over the nodes (ceil(B/N) per node, examples/cifar10.lua:36-37).  Each epoch:
train on this node's partition (label-uniform sampler, :53-71), all-reduce the
training confusion matrix (:203), ``synchronizeParameters`` (:208), evaluate
the test partition (:213-231) and all-reduce the test confusion matrix (:234).

MI355X path (``--cuda``): the dataset partition lives in HBM and the step is
the hand-written HIP executor (``--backend hip``, default) or PyTorch/MIOpen
ops (``--backend torch``), captured in a hipGraph.  With the HIP executor the
epoch runs on the same fast path as bench.py: a device-side label-uniform
sampler (``DeviceLoader``) whose batch is gathered + normalised inside the
step, ``trainer.run`` replaying unrolled multi-step graphs, and the
every-sample training confusion matrix updated by a kernel captured in the
step (``trainer.step_hooks``).  Without the dataset files (``--data`` directory with
the CIFAR-10 binary release) synthetic CIFAR-shaped data is used.

    python -m torch_distlearn_amd.launch --nproc 2 examples/cifar10.py --epochs 1
"""
import argparse
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torch_distlearn_amd import LocalhostTree  # noqa: E402
from torch_distlearn_amd.checkpoint import results_dir, resume_trainer, save_trainer  # noqa: E402
from torch_distlearn_amd.data import Dataset, DeviceLoader  # noqa: E402
from torch_distlearn_amd.engine import DataParallelTrainer  # noqa: E402
from torch_distlearn_amd.launch import (add_checkpoint_flags, add_node_flags, device_of, node_opts,  # noqa: E402
                                        quiet_unless_root)
from torch_distlearn_amd.models import CifarConvNet  # noqa: E402
from torch_distlearn_amd.utils.metrics import ConfusionMatrix, JsonlMetrics  # noqa: E402

CLASSES = ["airplane", "automobile", "bird", "cat", "deer", "dog", "frog", "horse", "ship", "truck"]


def main():
    ap = add_node_flags(argparse.ArgumentParser(description=__doc__.split("\n\n")[0]), batch=32, lr=0.1)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--maxSteps", type=int, default=0, help="stop each epoch after this many steps (0 = all)")
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"])
    ap.add_argument("--data", default=None, help="directory with the CIFAR-10 binary release (optional)")
    ap.add_argument("--trainSize", type=int, default=50000, help="synthetic train set size")
    ap.add_argument("--testSize", type=int, default=10000, help="synthetic test set size")
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--unroll", type=int, default=16, help="steps per replayed hipGraph (HIP fast path)")
    ap.add_argument("--metrics", default=None, help="JSON-lines metrics file (node 1)")
    add_checkpoint_flags(ap)
    opt = ap.parse_args()
    node_opts(opt)
    dev = device_of(opt)
    tree = LocalhostTree(opt.nodeIndex, opt.numNodes, port=opt.port, device=dev)
    quiet_unless_root(opt.nodeIndex)

    per_node = math.ceil(opt.batchSize / opt.numNodes)  # cifar10.lua:36
    train = Dataset("cifar10", opt.nodeIndex, opt.numNodes, train=True, root=opt.data, synthetic_size=opt.trainSize,
                    device=dev)
    test = Dataset("cifar10", opt.nodeIndex, opt.numNodes, train=False, root=opt.data, synthetic_size=opt.testSize,
                   device=dev)
    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    backend = opt.backend if dev.type == "cuda" else "torch"
    graph = bool(opt.graph) and dev.type == "cuda"
    fast = backend == "hip" and graph  # bench.py's path: device sampler + unrolled graph replays
    if fast:
        train_b = DeviceLoader(train, "label-uniform", per_node, seed=opt.seed + opt.nodeIndex)
    else:
        train_b = train.sampledBatcher("label-uniform", per_node, dtype=dt, seed=opt.seed + opt.nodeIndex)
    test_b = test.sampledBatcher("linear", per_node, dtype=dt)

    torch.manual_seed(0)  # same init on all nodes (cifar10.lua:105)
    model = CifarConvNet(seed=0).to(dev)
    trainer = DataParallelTrainer(model, tree, lr=opt.learningRate, backend=backend, compute_dtype=dt,
                                  graph=graph, max_batch=per_node)
    first = 1
    if opt.resume:
        st = resume_trainer(results_dir(opt.save, opt.resultsRoot), trainer)
        train_b.skip(int(st["node/drawn"][opt.nodeIndex - 1]))
        first = int(st["epoch"]) + 1
        print(f"resumed from {opt.resultsRoot}/{opt.save} after epoch {first - 1}")
    else:
        trainer.synchronize_parameters()  # cifar10.lua:139
    conf = ConfusionMatrix(CLASSES, device=dev)
    log = JsonlMetrics(opt.metrics, rank=opt.nodeIndex - 1)
    if fast:
        # every training sample enters the matrix (cifar10.lua:194-196): one
        # argmax+histogram kernel inside every captured step
        trainer.step_hooks.append(conf.add)
        trainer.prepare(train_b, opt.unroll)  # all captures happen here, before any timed epoch

    for epoch in range(first, opt.epochs + 1):
        conf.zero()
        nb = train_b.numBatches() if not opt.maxSteps else min(opt.maxSteps, train_b.numBatches())
        t0 = time.perf_counter()
        if fast:
            loss = trainer.run(train_b, nb, unroll=opt.unroll)
        else:
            for i in range(nb):
                x, y = train_b.getBatch()
                loss = trainer.step(x, y)
                # every training sample enters the matrix (cifar10.lua:194-196); on the GPU
                # this is one argmax+histogram kernel per step, no host sync
                conf.add(trainer.last_logits(), y)
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt_s = time.perf_counter() - t0
        conf.allReduce(tree)  # cifar10.lua:203
        path = f"unrolled hipGraphs x{opt.unroll}, {trainer.captures} captures" if fast else "step-by-step"
        print(f"Epoch {epoch}: train loss {float(loss):.4f}  {nb * per_node * opt.numNodes / dt_s:.0f} img/s "
              f"({nb} steps of {per_node} per node; {path})")
        print(conf)
        trainer.synchronize()  # cifar10.lua:208
        conf.zero()
        ntb = test_b.numBatches() if not opt.maxSteps else min(opt.maxSteps, test_b.numBatches())
        test_b.reset()
        for _ in range(ntb):
            x, y = test_b.getBatch()
            conf.add(trainer.predict(x), y)
        conf.allReduce(tree)  # cifar10.lua:234
        print(f"Epoch {epoch}: test accuracy {100 * conf.totalValid:.2f}%")
        log.log(epoch=epoch, loss=float(loss), images_per_s=nb * per_node * opt.numNodes / dt_s,
                test_acc=conf.totalValid)
        if opt.save:
            save_trainer(results_dir(opt.save, opt.resultsRoot), trainer, epoch, per_node={"drawn": train_b.drawn})
    tree.comm.barrier()


if __name__ == "__main__":
    main()
