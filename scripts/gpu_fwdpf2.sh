#!/bin/bash
# confirm: 4-stage fwd/dgrad with fragment prefetch (new default) vs the old 3-stage loop; wgrad 5 stages
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|assert" gpurun_out/pytest_iter.log | tail -8
[ $rc -ne 0 ] && exit 1
for r in 1 2 3; do
  for cfg in "DISTLEARN_NOP=1" "DISTLEARN_FWD_PF=0 DISTLEARN_FWD_STAGES=3 DISTLEARN_DGRAD_STAGES=3" "DISTLEARN_WGRAD_STAGES=5"; do
    out=$(env $cfg timeout -k 5 120 python bench.py --steps 600 --warmup 24 2>gpurun_out/ab_err.log) || { echo "bench failed ($cfg)"; tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "$cfg $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  done
done | tee gpurun_out/ab_fwdpf2.txt
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
rm -rf gpurun_out/prof
cat gpurun_out/timeline.txt
echo ALLDONE
