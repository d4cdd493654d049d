#!/bin/bash
# CIFAR kernel iteration: numerics tests of the touched kernels, 2x 600-step bench, step timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py tests/kernels/test_flat_ops_gpu.py} -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_iter.log | tail -8
[ $rc -ne 0 ] && exit 1
for r in 1 2; do
  timeout -k 10 120 python bench.py --steps 600 --warmup 24 > gpurun_out/b$r.log 2>&1 || exit 1
  tail -1 gpurun_out/b$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["ms_per_step"], d["value"], d["final_loss"])'
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
rm -rf gpurun_out/prof
cat gpurun_out/timeline.txt
echo ALLDONE
