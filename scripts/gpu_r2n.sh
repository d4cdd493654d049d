#!/bin/bash
# ResNet-50 kernel profile of the timed steps only (after MIOpen's solver search)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 -- python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/prof_r50.log 2>&1 || exit 1
python scripts/prof_summary.py gpurun_out/prof_r50 --steps 10 --top 70 --last-ms 290 --marker sgd_kernel > gpurun_out/r50_kernels.txt 2>&1 || true
rm -rf gpurun_out/prof_r50
tail -1 gpurun_out/prof_r50.log | cut -c1-200
