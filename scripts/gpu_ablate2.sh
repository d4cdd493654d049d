#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for ab in 0 31 95 127 32; do
  echo "== wablate $ab"
  timeout -k 10 120 python scripts/bench_conv.py --only wgrad --iters 40 --wablate $ab || exit 1
done > gpurun_out/wgrad_ablate2.txt 2>&1
grep -v amdgpu.ids gpurun_out/wgrad_ablate2.txt
echo ALLDONE
