#!/bin/bash
# A/B of one executor knob on the headline bench, runs interleaved in one call
# (box-to-box variation is larger than most effects):
#   scripts/ab_bench.sh <ENV_VAR> "<v1> <v2>" [rounds] [extra bench args...]
set -o pipefail
var=$1; vals=$2; rounds=${3:-3}; shift 3 2>/dev/null
mkdir -p gpurun_out
for r in $(seq "$rounds"); do
  for v in $vals; do
    out=$(env "$var=$v" timeout -k 5 120 python bench.py --steps 600 --warmup 24 "$@" 2>gpurun_out/ab_err.log) || { echo "bench failed ($var=$v)"; tail -5 gpurun_out/ab_err.log; exit 1; }
    echo "$var=$v $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["final_loss"])')"
  done
done
