#!/bin/bash
# EA unrolled graphs (tests + A/B unroll 1 vs 8) and the region images-mode A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/pytest_ea.log python -u -m pytest tests/kernels/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_ea.log && ! grep -q "failed\|error" gpurun_out/pytest_ea.log || { echo "TESTS FAILED"; exit 1; }
bash scripts/ab_bench.sh DISTLEARN_UNROLL "1 8" 2 --algo ea > gpurun_out/ab_ea_unroll.txt 2>&1 || exit 1
cat gpurun_out/ab_ea_unroll.txt
bash scripts/ab_bench.sh DISTLEARN_REGION "1 2" 2 > gpurun_out/ab_region.txt 2>&1 || exit 1
cat gpurun_out/ab_region.txt
echo ALLDONE
