#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_resnet_gpu.py tests/kernels/test_resnet_strided_gpu.py tests/kernels/test_conv_resnet_gpu.py tests/kernels/test_resnet_bn_dgrad_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_sw.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_sw.log
[ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in 1 0; do
    out=$(DISTLEARN_RESNET_STATS_WAVE=$v timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 2>gpurun_out/ab_err.log) || { tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "STATS_WAVE=$v $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  done
done > gpurun_out/ab_swave.txt
cat gpurun_out/ab_swave.txt
echo ALLDONE
