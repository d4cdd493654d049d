#!/bin/bash
# First-layer conv with the bank-conflict-free weight panel: tests, phase stamps,
# kernel durations in the step, LDS conflict counters.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/c8_tests.log python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
$S 120 gpurun_out/c8_stamp.log python scripts/stamp_c8.py 128 || exit 1
$S 240 gpurun_out/c8_prof.log rocprofv3 --kernel-trace --stats -d gpurun_out/c8prof -o run -- python bench.py --steps 30 --warmup 4 || exit 1
$S 120 gpurun_out/c8_pmc.log rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/c8pmc -o run -- python scripts/stamp_c8.py 128 || exit 1
$S 200 gpurun_out/c8_bench.log python bench.py || exit 1
echo ALLDONE
