#!/bin/bash
# BN kernel tuning A/B: per-shape BN microbench for each (apply rows, reduce
# threads) setting, BN GPU tests, then interleaved ResNet-50 steps.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for t in 2,256 4,256 4,512 4,1024 2,1024; do
  BN_TUNE=$t $S 120 gpurun_out/bn_$t.log python scripts/bench_bn.py || exit 1
done
$S 300 gpurun_out/pytest_bn.log python -u -m pytest tests/kernels/test_resnet_gpu.py tests/kernels/test_resnet_bn_dgrad_gpu.py tests/kernels/test_resnet_strided_gpu.py tests/kernels/test_conv_resnet_gpu.py -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2; do
  for t in 2,256 4,1024; do
    DISTLEARN_BN_TUNE=$t $S 300 gpurun_out/r50_${t}_$rep.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
  done
done
grep -h '"metric"' gpurun_out/r50_*.log | python -c "import sys,json; [print(json.loads(l)['ms_per_step']) for l in sys.stdin]"
echo ALLDONE
