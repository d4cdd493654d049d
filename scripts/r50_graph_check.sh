#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 gpurun_out/r50_graph.log python bench.py --model resnet50 --steps 40 --warmup 5 --graph 1 || exit 1
$S 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
echo ALLDONE
