#!/bin/bash
# Round-end rehearsal: smoke, the whole GPU test tier, headline bench, CIFAR step timeline, ResNet-50 bench + kernels
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread > gpurun_out/pytest_all.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" gpurun_out/pytest_all.log | tail -15
[ $rc -ge 124 ] && exit 1
timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final.log 2>&1 || exit 1
tail -1 gpurun_out/bench_final.log
echo ALLDONE
