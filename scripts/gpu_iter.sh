#!/bin/bash
# CIFAR iteration: convnet/engine GPU tests, 600-step bench x2, kernel timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/pytest_iter.log python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_iter.log && ! grep -q "failed\|error" gpurun_out/pytest_iter.log || { echo "TESTS FAILED"; exit 1; }
bash scripts/ab_bench.sh ${ABVAR:-DISTLEARN_NOP} "${ABVALS:-1}" ${ABROUNDS:-2} > gpurun_out/ab_iter.txt 2>&1 || exit 1
cat gpurun_out/ab_iter.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
rm -rf gpurun_out/prof
echo ALLDONE
