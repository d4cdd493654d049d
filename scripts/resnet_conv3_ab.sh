#!/bin/bash
# ResNet-50: 3x3 stride-1 convs on the HIP kernels up to H = 28 (default) vs also the 56x56 stage
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for hw in 28 56; do
    out=$(DISTLEARN_RESNET_CONV3_MAX_HW=$hw timeout -k 10 300 python bench.py --model resnet50 --steps 30 --warmup 6 2>gpurun_out/r50_err.log) || { echo "bench failed hw=$hw"; tail -5 gpurun_out/r50_err.log; exit 1; }
    echo "MAX_HW=$hw $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')" | tee -a gpurun_out/r50_conv3_ab.txt
  done
done
echo ALLDONE
