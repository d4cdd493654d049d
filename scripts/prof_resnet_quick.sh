#!/bin/bash
# ResNet-50: GPU tests of the ResNet kernels, bench, kernel summary of the timed steps
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
S=scripts/gpu_step.sh
$S 300 gpurun_out/r50_tests.log python -u -m pytest tests/kernels/test_resnet_gpu.py tests/kernels/test_conv_resnet_gpu.py -x -q --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r50_tests.log && ! grep -q "failed\|error" gpurun_out/r50_tests.log || { echo "TESTS FAILED"; exit 1; }
$S 300 gpurun_out/r50_bench.log python bench.py --model resnet50 --steps 30 --warmup 6 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 -- python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/prof_r50.log 2>&1 || exit 1
python scripts/prof_summary.py gpurun_out/prof_r50 --top 60 --last-ms 290 --marker sgd_kernel > gpurun_out/r50_kernels.txt 2>&1 || true
rm -rf gpurun_out/prof_r50
echo ALLDONE
