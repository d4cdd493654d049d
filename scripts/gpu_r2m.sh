#!/bin/bash
# CIFAR step: fresh mode-0 timeline + A/B of the streaming-kernel ring stages / waves
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
[ -n "$NOPROF" ] || timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
[ -n "$NOPROF" ] || python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
rm -rf gpurun_out/prof
for cfg in ${CFGS:-"X=0" "DISTLEARN_UNROLL=16" "DISTLEARN_UNROLL=32" "X=1" "DISTLEARN_UNROLL=16"}; do
  env $cfg timeout -k 10 120 python bench.py --steps 400 --warmup 20 > gpurun_out/ab.json 2> gpurun_out/ab.err || exit 1
  echo "$cfg $(tail -1 gpurun_out/ab.json | python -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"], d["final_loss"])')" | tee -a gpurun_out/ab.txt
done
