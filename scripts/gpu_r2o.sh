#!/bin/bash
# ResNet-50 kernel profiles with the 3x3 convs on MIOpen (0) vs the HIP kernels (28)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for hw in 0 28; do
  DISTLEARN_RESNET_CONV3_MAX_HW=$hw timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$hw -o r50 -- python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/prof_$hw.log 2>&1 || exit 1
  python scripts/prof_summary.py gpurun_out/prof_$hw --top 80 --last-ms 290 --marker sgd_kernel > gpurun_out/r50_k_$hw.txt 2>&1 || true
  rm -rf gpurun_out/prof_$hw
done
