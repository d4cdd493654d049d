#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
tail -8 gpurun_out/pytest_new.log
[ $rc -ge 124 ] && exit 1
bash scripts/ab_bench.sh DISTLEARN_HEAD_REDUCE "1 0" 2 > gpurun_out/ab_head_reduce.txt 2>&1 || exit 1
bash scripts/ab_bench.sh DISTLEARN_DGRAD_BNRED "1 0" 2 > gpurun_out/ab_dgrad_bnred.txt 2>&1 || exit 1
cat gpurun_out/ab_dgrad_bnred.txt
cat gpurun_out/ab_head_reduce.txt
bash scripts/gpu_regime.sh || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
rm -rf gpurun_out/prof
cat gpurun_out/timeline.txt
echo ALLDONE
