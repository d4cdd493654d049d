#!/bin/bash
# 256x128 / 32-row-step wgrad tile (tile 4): numerics, microbench at several split counts, end-to-end A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -k "dgrad_wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|assert" gpurun_out/pytest_iter.log | tail -8
[ $rc -ne 0 ] && exit 1
{
for r in 1 2; do
  echo "== wgrad3 tile 2 split 5"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad3 --wtile 2 --wsplits 5 2>&1 | grep -E "wgrad" || exit 1
  for sp in 5 8 10; do echo "== wgrad3 tile 4 split $sp"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad3 --wtile 4 --wsplits $sp 2>&1 | grep -E "wgrad" || exit 1; done
  echo "== wgrad4 tile 2 split 1"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad4 --wtile 2 --wsplits 1 2>&1 | grep -E "wgrad" || exit 1
  for sp in 1 2 3; do echo "== wgrad4 tile 4 split $sp"; timeout -k 10 60 python scripts/bench_conv.py --only wgrad4 --wtile 4 --wsplits $sp 2>&1 | grep -E "wgrad" || exit 1; done
done
} > gpurun_out/wtile_micro.txt 2>&1
cat gpurun_out/wtile_micro.txt
bash scripts/ab_bench.sh DISTLEARN_WGRAD_TILE "2 4" 2 > gpurun_out/ab_wtile.txt 2>&1 || { cat gpurun_out/ab_wtile.txt; exit 1; }
cat gpurun_out/ab_wtile.txt
echo ALLDONE
