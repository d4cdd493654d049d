#!/bin/bash
# wgrad main-loop ablation on the CIFAR shapes; BN-dgrad (BNR 2/3) tests + ResNet A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ab in 0 1 2 4 3 6 7; do
  echo "== wablate $ab"
  timeout -k 10 120 python scripts/bench_conv.py --only wgrad --iters 40 --wablate $ab || exit 1
done > gpurun_out/wgrad_ablate.txt 2>&1
cat gpurun_out/wgrad_ablate.txt
timeout -k 10 300 python -u -m pytest tests/kernels/test_resnet_bn_dgrad_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_bnd.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_bnd.log
[ $rc -ne 0 ] && exit 1
for r in 1 2; do
  for v in 1 0; do
    out=$(DISTLEARN_RESNET_BN_DGRAD=$v timeout -k 10 200 python bench.py --model resnet50 --steps 20 --warmup 5 2>gpurun_out/ab_err.log) || { tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "BN_DGRAD=$v $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  done
done > gpurun_out/ab_r50_bn_dgrad3.txt
cat gpurun_out/ab_r50_bn_dgrad3.txt
echo ALLDONE
