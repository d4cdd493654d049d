#!/bin/bash
# Interleaved A/B of one environment knob on the driver-form bench:
#   scripts/ab_env.sh VAR "v1 v2" ROUNDS [extra bench args...]
# Each run is one `bench.py --gpus 1 --steps 20 --warmup 5` (the driver's
# command) unless extra args are given; prints "VAR=v ms/step" lines.
var=$1; vals=$2; rounds=$3; shift 3
args="$@"
[ -z "$args" ] && args="--gpus 1 --steps 20 --warmup 5"
for r in $(seq 1 $rounds); do
  for v in $vals; do
    out=$(env $var=$v timeout -k 10 120 python bench.py $args 2>/dev/null | grep '^{' | tail -1)
    rc=$?
    ms=$(echo "$out" | python -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])" 2>/dev/null)
    echo "$var=$v round=$r ms_per_step=$ms"
    [ -z "$ms" ] && { echo "run failed"; exit 1; }
  done
done
