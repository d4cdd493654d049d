#!/bin/bash
# (record of a finished A/B: its DISTLEARN_AB_* toggles were removed when the result was adopted)
# Layer-3 dgrad on position-major tiles: 2 vs 4 splits (posm=2), vs pixel-major 2 splits.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "2 4" "2 3"; do
  set -- $cfg
  DISTLEARN_AB_POSM=$1 DISTLEARN_AB_D3S=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/posm8b_prof_$1_$2 -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/posm8b_prof.log 2>&1 || { tail -20 gpurun_out/posm8b_prof.log; exit 1; }
done
: > gpurun_out/posm8b_ab.txt
for r in 1 2 3 4 5; do
  for cfg in "2 2" "2 4" "1 2" "1 2" "2 4" "2 2"; do
    set -- $cfg
    DISTLEARN_AB_POSM=$1 DISTLEARN_AB_D3S=$2 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/posm8b_run.log 2>&1 || { tail -5 gpurun_out/posm8b_run.log; exit 1; }
    echo "posm=$1 d3s=$2 round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/posm8b_run.log)" | tee -a gpurun_out/posm8b_ab.txt
  done
done
echo ALLDONE
