#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/bench_barrier.py > gpurun_out/barrier.txt 2>&1; rc=$?
cat gpurun_out/barrier.txt
[ $rc -ne 0 ] && exit 1
timeout -k 10 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -x -q -k "wgrad" --timeout 120 --timeout-method thread 2>&1 | tail -2
for r in 1 2; do for ws in 1 0; do echo "== wstage $ws"; timeout -k 10 120 python scripts/bench_conv.py --only wgrad --iters 40 --wstage $ws 2>&1 | grep wgrad || exit 1; done; done
echo ALLDONE
