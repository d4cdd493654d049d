#!/bin/bash
# 4 local nodes, AllReduceEA tau=10 alpha=0.2 (reference: examples/mnist-ea.sh)
cd "$(dirname "$0")/.." && python -m torch_distlearn_amd.launch --nproc "${N:-4}" examples/mnist_ea.py "$@"
