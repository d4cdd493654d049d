#!/bin/bash
# Quick GPU iteration: GPU tests (optionally filtered), 1-GPU bench, kernel
# timeline of one steady-state step.   usage: gpu_quick.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
K=${1:-}
$S 400 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${K:+-k "$K"} || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q "failed\|error" gpurun_out/pytest_gpu.log || { echo "TESTS FAILED"; exit 1; }
$S 180 gpurun_out/bench_sgd.log python bench.py --steps 400 --warmup 24 || exit 1
$S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
python scripts/prof_summary.py gpurun_out/prof --steps 64 --top 30 > gpurun_out/kernels.txt 2>&1
echo ALLDONE
