#!/bin/bash
# rocprofv3 kernel stats of the ResNet-50 (BASELINE config 5) bench step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/rocprof_r50.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o run -- python bench.py --model resnet50 --steps 10 --warmup 3 || exit 1
echo ALLDONE
