#!/bin/bash
# ResNet-50 BN sums from the dgrad epilogue: tests, A/B, kernel stats; CIFAR split-K tile A/B.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_resnet_bn_dgrad_gpu.py tests/kernels/test_resnet_strided_gpu.py tests/kernels/test_resnet_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_bnd.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_bnd.log
[ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in 1 0; do
    out=$(DISTLEARN_RESNET_BN_DGRAD=$v timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 2>gpurun_out/ab_err.log) || { tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "BN_DGRAD=$v $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  done
done > gpurun_out/ab_r50_bn_dgrad.txt
cat gpurun_out/ab_r50_bn_dgrad.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 -- python bench.py --model resnet50 --steps 10 --warmup 5 > gpurun_out/prof_r50.log 2>&1 || exit 1
python scripts/prof_summary.py gpurun_out/prof_r50 --top 60 --last-ms 290 --marker sgd_kernel > gpurun_out/r50_kernels.txt 2>&1 || true
rm -rf gpurun_out/prof_r50
head -30 gpurun_out/r50_kernels.txt
bash scripts/ab_bench.sh DISTLEARN_SPLIT_128x64 "0 1" 2 > gpurun_out/ab_split128x64.txt 2>&1 || exit 1
cat gpurun_out/ab_split128x64.txt
echo ALLDONE
