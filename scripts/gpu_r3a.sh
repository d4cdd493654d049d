#!/bin/bash
# Round-3 check: smoke, whole GPU test tier, headline bench, barrier prices, CIFAR step timeline
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_all.log | tail -15
[ $rc -ne 0 ] && exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || exit 1
tail -1 gpurun_out/bench_final.log
timeout -k 10 60 python scripts/bench_barrier.py > gpurun_out/barrier.txt 2>&1 || exit 1
cat gpurun_out/barrier.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
rm -rf gpurun_out/prof
tail -3 gpurun_out/timeline.txt
echo ALLDONE
