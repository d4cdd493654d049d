#!/usr/bin/env python3
"""MNIST convnet trained with AllReduceEA (reference: examples/mnist-ea.lua).

Elastic averaging every ``--tau`` steps with moving rate ``--alpha``
(reference: tau 10, alpha 0.2, examples/mnist-ea.lua:18); SGD step, then
``averageParameters`` (:103-110); ``synchronizeCenter`` at epoch end (:121).

    python -m torch_distlearn_amd.launch --nproc 4 examples/mnist_ea.py --epochs 1
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mnist import parser, run  # noqa: E402

if __name__ == "__main__":
    ap = parser(__doc__.split("\n\n")[0])
    ap.add_argument("--tau", type=int, default=10)
    ap.add_argument("--alpha", type=float, default=0.2)
    run(ap.parse_args(), "ea")
