#!/bin/bash
# 256x128 wgrad tile (no fragment prefetch): microbench at the executor's split counts, end-to-end A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
{
for r in 1 2; do
  for sp in 5 10; do echo "== wgrad3 tile 2 split $sp"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad3 --wtile 2 --wsplits $sp 2>&1 | grep -E "wgrad" || exit 1; done
  for sp in 8 10 16; do echo "== wgrad3 tile 3 split $sp"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad3 --wtile 3 --wsplits $sp 2>&1 | grep -E "wgrad" || exit 1; done
  for sp in 2 3 4; do echo "== wgrad4 tile 3 split $sp"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad4 --wtile 3 --wsplits $sp 2>&1 | grep -E "wgrad" || exit 1; done
done
} > gpurun_out/wtile_micro.txt 2>&1
cat gpurun_out/wtile_micro.txt
bash scripts/ab_bench.sh DISTLEARN_WGRAD_256 "0 1" 2 > gpurun_out/ab_wtile.txt 2>&1 || { cat gpurun_out/ab_wtile.txt; exit 1; }
cat gpurun_out/ab_wtile.txt
echo ALLDONE
