#!/bin/bash
# ResNet BN backward apply with folded coefficients: BN microbench, ResNet GPU tests, ResNet bench x2.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/pytest_r50.log python -u -m pytest tests/kernels/test_resnet_gpu.py tests/kernels/test_resnet_bn_dgrad_gpu.py tests/kernels/test_resnet_strided_gpu.py tests/kernels/test_conv_resnet_gpu.py -x -q --timeout 200 --timeout-method thread || exit 1
BN_TUNE=4,256 $S 120 gpurun_out/bn_4,256.log python scripts/bench_bn.py || exit 1
BN_TUNE=2,256 $S 120 gpurun_out/bn_2,256.log python scripts/bench_bn.py || exit 1
$S 300 gpurun_out/r50_1.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
$S 300 gpurun_out/r50_2.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
for f in gpurun_out/r50_?.log; do
  echo "$f $(grep -h '"metric"' $f | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
echo ALLDONE
