#!/bin/bash
# Multi-node step configuration on one GPU (bench.py --nworld-path): the old
# N>1 chain (slab_reduce per layer, a prep launch per step) vs the fused one
# (slab sums on the dgrad / one merged launch, the update preparing the next
# step), interleaved, each with both overlap policies timed by select_policy;
# then both policies forced with 32 CUs held by RCCL-footprint workgroups.
#   scripts/nworld_ab.sh [rounds] [out]
set -o pipefail
rounds=${1:-2}; out=${2:-gpurun_out/r5_nworld_ab.txt}
mkdir -p gpurun_out
: > "$out"
one() {  # label, env..., -- bench args
  local label=$1; shift
  local envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  local o
  o=$(env "${envs[@]}" timeout -k 5 150 python bench.py --steps 600 --warmup 24 --nworld-path 1 "$@" 2>gpurun_out/nworld_err.log) \
    || { echo "bench failed ($label)" | tee -a "$out"; tail -20 gpurun_out/nworld_err.log | tee -a "$out"; exit 1; }
  echo "$label $(echo "$o" | tail -1 | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(d["ms_per_step"], d["value"], d["final_loss"], "policy", json.dumps(c.get("policy")), "fused", json.dumps(c["nworld_path"]["fused_slab_reduce"]))')" | tee -a "$out"
}
for r in $(seq "$rounds"); do
  one old DISTLEARN_FUSE_REDUCE=0 DISTLEARN_PREP_NEXT=0 --
  one fused DISTLEARN_FUSE_REDUCE=1 DISTLEARN_PREP_NEXT=1 --
done
for pol in full reserve; do
  one "old_hold32_$pol" DISTLEARN_POLICY=$pol DISTLEARN_FUSE_REDUCE=0 DISTLEARN_PREP_NEXT=0 -- --hold-cus 32
  one "fused_hold32_$pol" DISTLEARN_POLICY=$pol -- --hold-cus 32
done
