#!/bin/bash
# Cost of the bucketed all-reduce's stream fork/join inside the replayed graph at
# N = 1: collectives forced through RCCL at world 1 (DISTLEARN_RCCL_WORLD1=1, a
# self all-reduce per bucket) for 1, 2-3 buckets, vs no collective.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
for rep in 1 2; do
  $S 120 gpurun_out/fc_none_$rep.log python bench.py --steps 20 --warmup 5 || exit 1
  for mb in 1 4 64; do
    DISTLEARN_RCCL_WORLD1=1 $S 120 gpurun_out/fc_rccl_${mb}_$rep.log python bench.py --steps 20 --warmup 5 --bucket-mb $mb || exit 1
  done
  DISTLEARN_RCCL_WORLD1=1 $S 120 gpurun_out/fc_rccl_1_nooverlap_$rep.log python bench.py --steps 20 --warmup 5 --overlap 0 || exit 1
done
DISTLEARN_RCCL_WORLD1=1 $S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline_rccl1.txt 2>&1
for f in gpurun_out/fc_*.log; do
  echo "$f $(grep -h '"metric"' $f | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
echo ALLDONE
