#!/bin/bash
# wgrad with asm LDS-DMA (no compiler vmcnt(0) before the transposed reads): tests, micro-bench sweep, benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_conv_ex_gpu.py tests/kernels/test_conv_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_wg.log 2>&1
rc=$?
tail -4 gpurun_out/pytest_wg.log
[ $rc -ne 0 ] && exit 1
for st in "3,0" "3,3" "3,4"; do
  for pf in -1 0 1; do
    echo "== stages $st pf $pf"
    timeout -k 10 120 python scripts/bench_conv.py --only wgrad --iters 40 --stages $st --wpf $pf 2>&1 | grep wgrad || exit 1
  done
done > gpurun_out/wgrad_sweep.txt 2>&1
cat gpurun_out/wgrad_sweep.txt
timeout -k 10 120 python bench.py > gpurun_out/bench_c.log 2>&1 || exit 1
tail -1 gpurun_out/bench_c.log
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_r50.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r50.log
echo ALLDONE
