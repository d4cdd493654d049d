#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_conv_ex_gpu.py tests/kernels/test_conv_resnet_gpu.py -x -q -k "wgrad or executor or resnet" --timeout 120 --timeout-method thread > gpurun_out/pytest_ws.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ws.log
[ $rc -ne 0 ] && exit 1
for r in 1 2; do for ws in 1 0; do
  echo "== wstage $ws"
  timeout -k 10 120 python scripts/bench_conv.py --only wgrad --iters 40 --wstage $ws 2>&1 | grep wgrad || exit 1
done; done > gpurun_out/wstage.txt 2>&1
cat gpurun_out/wstage.txt
echo ALLDONE
