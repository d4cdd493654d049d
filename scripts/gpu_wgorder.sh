#!/bin/bash
# wgrad main-loop order A/B: per-layer microbench, numerics, end-to-end interleaved bench
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 0 1 0 1; do
  echo "== worder $o"; timeout -k 10 120 python scripts/bench_conv.py --only wgrad --worder $o 2>&1 | grep wgrad || exit 1
done > gpurun_out/wgorder_micro.txt
cat gpurun_out/wgorder_micro.txt
timeout -k 10 400 python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_conv_ex_gpu.py tests/kernels/test_conv_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_iter.log | tail -8
[ $rc -ne 0 ] && exit 1
bash scripts/ab_bench.sh DISTLEARN_WGRAD_ORDER "0 1" 3 > gpurun_out/ab_wgorder.txt 2>&1 || { cat gpurun_out/ab_wgorder.txt; exit 1; }
cat gpurun_out/ab_wgorder.txt
echo ALLDONE
