#!/bin/bash
# Does the driver command (20 steps, 5 warm-up) read slower than 50-step runs
# because of the warm-up length?  Interleaved on one box.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/warm_ab.txt
for r in 1 2 3; do
  for cfg in "20 5" "20 50" "50 10" "200 10"; do
    set -- $cfg
    timeout -k 10 200 python bench.py --gpus 1 --steps $1 --warmup $2 > gpurun_out/warm_run.log 2>&1 || { tail -5 gpurun_out/warm_run.log; exit 1; }
    echo "steps=$1 warmup=$2 round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/warm_run.log)" | tee -a gpurun_out/warm_ab.txt
  done
done
echo ALLDONE
