#!/bin/bash
# (record of a finished A/B: its DISTLEARN_AB_* toggles were removed when the result was adopted)
# Pair-packed first layer on the 4-channel input (forward + weight gradient):
# GPU tests, a kernel profile and an interleaved step A/B against the
# channel-padded layer 1 (DISTLEARN_AB_PAIR1=0).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_convnet_gpu.py \
  -k "pair or padded or prep_step or matches_torch" > gpurun_out/pair2_tests.log 2>&1 || { tail -30 gpurun_out/pair2_tests.log; exit 1; }
tail -3 gpurun_out/pair2_tests.log
for v in 1 0; do
  DISTLEARN_AB_PAIR1=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pair2_prof$v -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/pair2_prof$v.log 2>&1 || { tail -20 gpurun_out/pair2_prof$v.log; exit 1; }
done
: > gpurun_out/pair2_ab.txt
for r in 1 2 3 4 5; do
  for v in 1 0 0 1; do
    DISTLEARN_AB_PAIR1=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/pair2_run.log 2>&1 || { tail -5 gpurun_out/pair2_run.log; exit 1; }
    echo "pair1=$v round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pair2_run.log)" | tee -a gpurun_out/pair2_ab.txt
  done
done
echo ALLDONE
