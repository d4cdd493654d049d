#!/bin/bash
# 128x128 weight-gradient tile on 4 waves (64x64 per wave, tile 3) vs 8 waves (tile 2).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_convnet_gpu.py \
  -k "dgrad_wgrad" > gpurun_out/wg4_tests.log 2>&1 || { tail -30 gpurun_out/wg4_tests.log; exit 1; }
tail -2 gpurun_out/wg4_tests.log
: > gpurun_out/wg4_bench.txt
for r in 1 2; do
  for t in 2 3; do
    timeout -k 10 120 python scripts/bench_conv.py --only wgrad --wtile $t --iters 100 >> gpurun_out/wg4_bench.txt 2>&1 || { tail -20 gpurun_out/wg4_bench.txt; exit 1; }
  done
done
cat gpurun_out/wg4_bench.txt
echo ALLDONE
