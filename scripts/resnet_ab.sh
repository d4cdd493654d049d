#!/bin/bash
# ResNet-50 (BASELINE config 5): BN tests, then BatchNorm mode A/B back to back
# on one box (mixed = MIOpen BN on bf16 + torch ReLU/add; hip = fused HIP BN).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/r50_tests.log python -u -m pytest tests/kernels/test_resnet_gpu.py -x -v --timeout 120 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/r50_tests.log && ! grep -q "failed" gpurun_out/r50_tests.log || { echo "tests failed"; exit 1; }
$S 200 gpurun_out/r50_bn_hip.log env DISTLEARN_RESNET_BN=hip python bench.py --model resnet50 --steps 30 --warmup 5 || exit 1
$S 200 gpurun_out/r50_bn_mixed.log env DISTLEARN_RESNET_BN=mixed python bench.py --model resnet50 --steps 30 --warmup 5 || exit 1
echo ALLDONE
