#!/bin/bash
# 4 local nodes, AllReduceSGD (reference: examples/mnist.sh)
cd "$(dirname "$0")/.." && python -m torch_distlearn_amd.launch --nproc "${N:-4}" examples/mnist.py "$@"
