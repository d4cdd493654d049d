#!/bin/bash
# (record of a finished A/B: its DISTLEARN_AB_* toggles were removed when the result was adopted)
# Position-major tiles (padding taps skipped) extended to the 8x8 layer-3
# dgrad: correctness check, kernel profile and interleaved step A/B.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
# (the one-off correctness check became POSM_SHAPES rows in tests/kernels/test_convnet_gpu.py)
for v in 1 2; do
  DISTLEARN_AB_POSM=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/posm8_prof$v -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/posm8_prof.log 2>&1 || { tail -20 gpurun_out/posm8_prof.log; exit 1; }
done
: > gpurun_out/posm8_ab.txt
for r in 1 2 3 4 5; do
  for v in 2 1 1 2; do
    DISTLEARN_AB_POSM=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/posm8_run.log 2>&1 || { tail -5 gpurun_out/posm8_run.log; exit 1; }
    echo "posm=$v round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/posm8_run.log)" | tee -a gpurun_out/posm8_ab.txt
  done
done
echo ALLDONE
