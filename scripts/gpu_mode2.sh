#!/bin/bash
# Reduction mode 2 (striped atomic BN rows): kernel/executor tests, interleaved
# A/B against mode 0 on the headline bench, kernel timeline of a mode-2 step.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/pytest_mode2.log python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "atomic or executor_matches or fused_finalize or head_pool or prep_zero" || exit 1
grep -q " passed" gpurun_out/pytest_mode2.log && ! grep -q "failed\|error" gpurun_out/pytest_mode2.log || { echo "TESTS FAILED"; exit 1; }
for R in ${ROWS:-16}; do
  DISTLEARN_REDUCE_ROWS=$R bash scripts/ab_bench.sh DISTLEARN_REDUCE_ATOMIC "0 2" 3 > gpurun_out/ab_mode2_r$R.txt 2>&1 || exit 1
  cat gpurun_out/ab_mode2_r$R.txt
done
DISTLEARN_REDUCE_ATOMIC=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof2 -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof2.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof2/run_results.db > gpurun_out/timeline_mode2.txt 2>&1
rm -rf gpurun_out/prof2
echo ALLDONE
