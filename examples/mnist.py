#!/usr/bin/env python3
"""MNIST convnet trained with AllReduceSGD (reference: examples/mnist.lua).

Per-node batch ``--batchSize`` (reference: 1, :33), lr 0.01 (:113), each node
trains on its partition with a permutation sampler (:26-40) -- partitions of
unequal length give nodes different step counts per epoch, which
``synchronizeParameters`` reconciles with the drain protocol (:129).  The
confusion matrix is all-reduced and printed every ``--printEvery`` steps
(:119-125).  ``--model mlp`` trains the 2-layer MLP of BASELINE config 1.

    python -m torch_distlearn_amd.launch --nproc 4 examples/mnist.py --epochs 1
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torch_distlearn_amd import LocalhostTree  # noqa: E402
from torch_distlearn_amd.checkpoint import results_dir, resume_trainer, save_trainer  # noqa: E402
from torch_distlearn_amd.data import Dataset  # noqa: E402
from torch_distlearn_amd.engine import DataParallelTrainer  # noqa: E402
from torch_distlearn_amd.launch import (add_checkpoint_flags, add_node_flags, device_of, node_opts,  # noqa: E402
                                        quiet_unless_root)
from torch_distlearn_amd.models import MnistConvNet, MnistMLP  # noqa: E402
from torch_distlearn_amd.utils.metrics import ConfusionMatrix  # noqa: E402


def build(opt, algo):
    node_opts(opt)
    dev = device_of(opt)
    tree = LocalhostTree(opt.nodeIndex, opt.numNodes, port=opt.port, device=dev)
    quiet_unless_root(opt.nodeIndex)
    ds = Dataset("mnist", opt.nodeIndex, opt.numNodes, train=True, root=opt.data, synthetic_size=opt.trainSize,
                 device=dev)
    dt = torch.bfloat16 if dev.type == "cuda" else torch.float32
    batcher = ds.sampledBatcher("permutation", opt.batchSize, dtype=dt, seed=opt.seed + opt.nodeIndex)
    torch.manual_seed(0)
    model = (MnistMLP(seed=0) if opt.model == "mlp" else MnistConvNet(seed=0)).to(dev)
    # --cuda: the convnet's whole step is one hand-written kernel (models/mnist_hip.py)
    backend = opt.backend if (dev.type == "cuda" and opt.model == "convnet") else "torch"
    trainer = DataParallelTrainer(model, tree, lr=opt.learningRate, algo=algo, tau=getattr(opt, "tau", 10),
                                  alpha=getattr(opt, "alpha", 0.2), backend=backend, compute_dtype=dt,
                                  graph=bool(opt.graph) and dev.type == "cuda" and algo == "sgd",
                                  max_batch=opt.batchSize)
    return tree, dev, batcher, model, trainer


def run(opt, algo="sgd"):
    tree, dev, batcher, model, trainer = build(opt, algo)
    first = 1
    if opt.resume:
        # Results/<save>/{Net, optState}: params, algorithm state, this node's sample stream
        st = resume_trainer(results_dir(opt.save, opt.resultsRoot), trainer)
        batcher.skip(int(st["node/drawn"][opt.nodeIndex - 1]))
        first = int(st["epoch"]) + 1
        print(f"resumed from {opt.resultsRoot}/{opt.save} after epoch {first - 1}")
    else:
        trainer.synchronize_parameters()
    conf = ConfusionMatrix(10, device=dev)
    step = 0
    for epoch in range(first, opt.epochs + 1):
        nb = batcher.numBatches() if not opt.maxSteps else min(opt.maxSteps, batcher.numBatches())
        # uneven partitions: the last node(s) may run one step less -> drain protocol at sync
        for _ in range(nb):
            x, y = batcher.getBatch()
            loss = trainer.step(x, y)
            conf.add(trainer.last_logits(), y)
            step += 1
        # the reference all-reduces the matrix every 1000 steps (mnist.lua:119-125); a collective
        # inside the loop requires equal step counts on every node, so it is done per epoch here
        conf.allReduce(tree)
        print(f"Epoch {epoch}: loss {float(loss):.4f}")
        print(conf)
        conf.zero()
        trainer.synchronize()
        if opt.save:
            save_trainer(results_dir(opt.save, opt.resultsRoot), trainer, epoch, per_node={"drawn": batcher.drawn})
    tree.comm.barrier()
    return trainer


def parser(desc, lr=0.01, batch=1):
    ap = add_node_flags(argparse.ArgumentParser(description=desc), batch=batch, lr=lr)
    ap.add_argument("--epochs", type=int, default=100)
    ap.add_argument("--maxSteps", type=int, default=0)
    ap.add_argument("--model", default="convnet", choices=["convnet", "mlp"])
    ap.add_argument("--data", default=None, help="directory with the MNIST idx files (optional)")
    ap.add_argument("--trainSize", type=int, default=60000)
    ap.add_argument("--graph", type=int, default=1)
    ap.add_argument("--backend", default="hip", choices=["hip", "torch"],
                    help="--cuda convnet: fused HIP step kernel (hip) or PyTorch ops (torch)")
    add_checkpoint_flags(ap)
    return ap


if __name__ == "__main__":
    run(parser(__doc__.split("\n\n")[0]).parse_args(), "sgd")
