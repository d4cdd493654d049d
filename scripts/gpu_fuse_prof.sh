#!/bin/bash
# kernel timelines of one steady-state CIFAR step with / without the fused split-K combine
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for F in 1 0; do
  DISTLEARN_FUSE_COMBINE=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$F -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof$F.log 2>&1 || { echo "rocprof $F failed"; tail -5 gpurun_out/rocprof$F.log; exit 1; }
  python scripts/prof_timeline.py gpurun_out/prof$F/run_results.db > gpurun_out/timeline$F.txt 2>&1
  rm -rf gpurun_out/prof$F
  echo "== fuse $F"; cat gpurun_out/timeline$F.txt
done
echo ALLDONE
