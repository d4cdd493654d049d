#!/bin/bash
# (record of a finished A/B: its DISTLEARN_AB_* toggles were removed when the result was adopted)
# Layer-1 weight-gradient split count on the pair-packed layout (256 = the
# plan, 128) vs the channel-padded layer 1, with 8-deep slab-reduce batches.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_convnet_gpu.py \
  -k "pair or padded or slab or matches_torch or deferred" > gpurun_out/pair3_tests.log 2>&1 || { tail -30 gpurun_out/pair3_tests.log; exit 1; }
tail -3 gpurun_out/pair3_tests.log
for cfg in "1 256" "1 128" "0 128"; do
  set -- $cfg
  DISTLEARN_AB_PAIR1=$1 DISTLEARN_AB_W1SPLITS=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pair3_prof_$1_$2 -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/pair3_prof.log 2>&1 || { tail -20 gpurun_out/pair3_prof.log; exit 1; }
done
: > gpurun_out/pair3_ab.txt
for r in 1 2 3 4 5; do
  for cfg in "1 256" "1 128" "0 128" "0 128" "1 128" "1 256"; do
    set -- $cfg
    DISTLEARN_AB_PAIR1=$1 DISTLEARN_AB_W1SPLITS=$2 timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/pair3_run.log 2>&1 || { tail -5 gpurun_out/pair3_run.log; exit 1; }
    echo "pair1=$1 w1splits=$2 round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/pair3_run.log)" | tee -a gpurun_out/pair3_ab.txt
  done
done
echo ALLDONE
