#!/bin/bash
# ResNet-50: hipGraph-captured step vs eager, same steps (loss trajectories must agree).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 gpurun_out/r50_eager40.log python bench.py --model resnet50 --steps 40 --warmup 5 --graph 0 || exit 1
$S 200 gpurun_out/r50_graph40.log python bench.py --model resnet50 --steps 40 --warmup 5 --graph 1 || exit 1
echo ALLDONE
