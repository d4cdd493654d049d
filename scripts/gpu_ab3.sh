#!/bin/bash
# re-A/B of the head BN-reduce fusion after the head rework
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/ab_bench.sh DISTLEARN_HEAD_REDUCE "1 0" 3 > gpurun_out/ab_head_reduce.txt 2>&1 || { cat gpurun_out/ab_head_reduce.txt; exit 1; }
cat gpurun_out/ab_head_reduce.txt
echo ALLDONE
