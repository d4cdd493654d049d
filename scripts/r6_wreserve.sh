#!/bin/bash
# The "wreserve" overlap policy (wgrad grids leave the RCCL channel cap of CUs
# free, dgrads keep 3 stages) on the world > 1 path, with and without 32 held CUs.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_engine_gpu.py \
  -k "policy" > gpurun_out/wres_tests.log 2>&1 || { tail -30 gpurun_out/wres_tests.log; exit 1; }
tail -2 gpurun_out/wres_tests.log
: > gpurun_out/wres.txt
for r in 1 2; do
  for cfg in "0 auto" "0 wreserve" "0 full" "32 wreserve" "32 full" "32 auto"; do
    set -- $cfg
    DISTLEARN_POLICY=$2 timeout -k 10 150 python bench.py --nworld-path 1 --hold-cus $1 > gpurun_out/wres_run.log 2>&1 || { tail -5 gpurun_out/wres_run.log; exit 1; }
    echo "hold=$1 policy=$2 round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wres_run.log | head -1) chosen=$(grep -o '"chosen": "[^"]*"' gpurun_out/wres_run.log | head -1)" | tee -a gpurun_out/wres.txt
  done
done
echo ALLDONE
