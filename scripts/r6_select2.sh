#!/bin/bash
# Two-pass policy selection on the world > 1 path (no CU held): chosen policy vs forced full.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_engine_gpu.py \
  -k "policy" > gpurun_out/sel2_tests.log 2>&1 || { tail -30 gpurun_out/sel2_tests.log; exit 1; }
tail -2 gpurun_out/sel2_tests.log
: > gpurun_out/sel2.txt
for r in 1 2 3; do
  for pol in auto full; do
    DISTLEARN_POLICY=$pol timeout -k 10 150 python bench.py --nworld-path 1 > gpurun_out/sel2_run.log 2>&1 || { tail -5 gpurun_out/sel2_run.log; exit 1; }
    echo "policy=$pol round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sel2_run.log | head -1) $(grep -o '"chosen": "[^"]*"' gpurun_out/sel2_run.log | head -1) $(grep -o '"ms_per_step": {[^}]*}' gpurun_out/sel2_run.log | head -1)" | tee -a gpurun_out/sel2.txt
  done
done
echo ALLDONE
