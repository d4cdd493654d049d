#!/bin/bash
# Full GPU tests with the mode-2 default, smoke, then R sweep of mode 2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 500 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed\|error" gpurun_out/pytest_gpu.log || { echo "TESTS FAILED"; exit 1; }
$S 180 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
bash scripts/ab_bench.sh DISTLEARN_REDUCE_ROWS "4 8 16 32" 2 > gpurun_out/ab_rows.txt 2>&1 || exit 1
cat gpurun_out/ab_rows.txt
$S 120 gpurun_out/bench_driver.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
echo ALLDONE
