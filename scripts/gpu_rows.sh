#!/bin/bash
# Striped BN accumulator rows (DISTLEARN_REDUCE_ROWS 8 vs 16) after the round-3 consumer-kernel changes.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for rep in 1 2 3; do
  for r in 16 8; do
    DISTLEARN_REDUCE_ROWS=$r $S 120 gpurun_out/rows${r}_$rep.log python bench.py --steps 400 --warmup 24 || exit 1
  done
done
for f in gpurun_out/rows*.log; do
  echo "$f $(grep -h '"metric"' $f | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
echo ALLDONE
