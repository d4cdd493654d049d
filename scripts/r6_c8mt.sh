#!/bin/bash
# (record of a finished A/B: its DISTLEARN_AB_* toggle was removed, the default kept)
# First-layer pair-packed forward: M tiles per workgroup 1 / 2 / 4 (set_conv_c8_mt).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in 2 4; do
  DISTLEARN_AB_C8MT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c8mt_prof$v -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/c8mt_prof.log 2>&1 || { tail -20 gpurun_out/c8mt_prof.log; exit 1; }
done
DISTLEARN_AB_C8MT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/c8mt_prof1 -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/c8mt_prof.log 2>&1 || { tail -20 gpurun_out/c8mt_prof.log; exit 1; }
: > gpurun_out/c8mt_ab.txt
for r in 1 2 3 4; do
  for v in 1 2 4 4 2 1; do
    DISTLEARN_AB_C8MT=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/c8mt_run.log 2>&1 || { tail -5 gpurun_out/c8mt_run.log; exit 1; }
    echo "c8mt=$v round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/c8mt_run.log)" | tee -a gpurun_out/c8mt_ab.txt
  done
done
echo ALLDONE
