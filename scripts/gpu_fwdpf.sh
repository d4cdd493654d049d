#!/bin/bash
# streaming fwd/dgrad fragment prefetch: bitwise test, microbench (stages x pf), end-to-end A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -k "prefetch_pipeline or fwd_and_stats or dgrad_wgrad" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed|assert" gpurun_out/pytest_iter.log | tail -8
[ $rc -ne 0 ] && exit 1
{
for st in 3 4; do for pf in 0 1; do
  echo "== stages $st pf $pf"; timeout -k 10 60 python scripts/bench_conv.py --stages $st,0 --fpf $pf --region 1 2>&1 | grep -E "fwd|dgrad" || exit 1
done; done
} > gpurun_out/fwdpf_micro.txt 2>&1
cat gpurun_out/fwdpf_micro.txt
for r in 1 2; do
  for cfg in "DISTLEARN_FWD_PF=0" "DISTLEARN_FWD_PF=1" "DISTLEARN_FWD_PF=1 DISTLEARN_FWD_STAGES=4 DISTLEARN_DGRAD_STAGES=4" "DISTLEARN_FWD_PF=0 DISTLEARN_FWD_STAGES=4 DISTLEARN_DGRAD_STAGES=4"; do
    out=$(env $cfg timeout -k 5 120 python bench.py --steps 600 --warmup 24 2>gpurun_out/ab_err.log) || { echo "bench failed ($cfg)"; tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "$cfg $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  done
done | tee gpurun_out/ab_fwdpf.txt
echo ALLDONE
