#!/bin/bash
# one node per GPU, RCCL over xGMI (reference: examples/cifar10-cuda.sh, 4 GPUs)
cd "$(dirname "$0")/.." && python -m torch_distlearn_amd.launch --nproc "${N:-4}" --gpus examples/cifar10.py "$@"
