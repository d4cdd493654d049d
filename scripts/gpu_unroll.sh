#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2 3; do
  for u in 16 20 32; do
    out=$(DISTLEARN_UNROLL=$u timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 2>/dev/null) || exit 1
    echo "unroll=$u steps=20 $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
  out=$(timeout -k 10 120 python bench.py --gpus 1 --steps 600 --warmup 24 2>/dev/null) || exit 1
  echo "unroll=16 steps=600 $(echo "$out" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done > gpurun_out/unroll_ab.txt
cat gpurun_out/unroll_ab.txt
echo ALLDONE
