#!/bin/bash
# ad-hoc GPU check: new kernel tests, ResNet-50 bench + kernel profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_resnet_strided_gpu.py tests/kernels/test_convnet_gpu.py tests/kernels/test_conv_resnet_gpu.py tests/kernels/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_new.log
[ $rc -ge 124 ] && exit 1
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r50_bench.log 2>&1 || { tail -20 gpurun_out/r50_bench.log; exit 1; }
tail -1 gpurun_out/r50_bench.log
DISTLEARN_RESNET_STRIDED=0 DISTLEARN_RESNET_HEAD=torch timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/r50_bench_old.log 2>&1 || { tail -20 gpurun_out/r50_bench_old.log; exit 1; }
tail -1 gpurun_out/r50_bench_old.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 -- python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/prof_r50.log 2>&1 || { tail -5 gpurun_out/prof_r50.log; exit 1; }
python scripts/prof_summary.py gpurun_out/prof_r50 --marker sgd_kernel --top 60 > gpurun_out/r50_kernels.txt 2>&1
rm -rf gpurun_out/prof_r50
head -40 gpurun_out/r50_kernels.txt

bash scripts/ab_bench.sh DISTLEARN_FWD_NOSPLIT64 "0 1" 2 > gpurun_out/ab_nosplit64.txt 2>&1 || exit 1
cat gpurun_out/ab_nosplit64.txt
echo ALLDONE
