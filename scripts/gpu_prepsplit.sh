#!/bin/bash
# How much of the prep launch is the dgrad weight transposes: one-step timeline
# with the transposes in their own launch (DISTLEARN_PREP_FORK=1, side stream).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
DISTLEARN_PREP_FORK=1 $S 240 gpurun_out/rocprof_fork.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fork -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof_fork/run_results.db > gpurun_out/timeline_fork.txt 2>&1
head -8 gpurun_out/timeline_fork.txt
echo ALLDONE
