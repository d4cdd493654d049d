#!/bin/bash
# Reduction-mode-1 check: convnet kernel numerics + engine tests, then bench in
# both modes back to back, then a kernel timeline of the new step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/pytest_gpu.log python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -x -q -rs --timeout 150 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed\| error" gpurun_out/pytest_gpu.log || { echo "TESTS FAILED"; exit 1; }
$S 120 gpurun_out/bench_m1_20.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 180 gpurun_out/bench_m1_400.log python bench.py --steps 400 --warmup 24 || exit 1
DISTLEARN_REDUCE_ATOMIC=0 $S 180 gpurun_out/bench_m0_400.log python bench.py --steps 400 --warmup 24 || exit 1
$S 180 gpurun_out/bench_m1_400b.log python bench.py --steps 400 --warmup 24 || exit 1
$S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
python scripts/prof_summary.py gpurun_out/prof --steps 64 --top 40 > gpurun_out/kernels.txt 2>&1
echo ALLDONE
