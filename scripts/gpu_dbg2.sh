#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_convnet_gpu.py -q --timeout 120 --timeout-method thread > gpurun_out/pytest_cn.log 2>&1
grep -E "FAILED|passed|failed" gpurun_out/pytest_cn.log | tail -30
echo ALLDONE
