#!/bin/bash
# 2 CPU nodes (reference: examples/cifar10.sh)
cd "$(dirname "$0")/.." && python -m torch_distlearn_amd.launch --nproc "${N:-2}" examples/cifar10.py "$@"
