#!/bin/bash
# Round-6 baseline: driver-form bench x2, and one-step kernel timelines at
# batch 128 / 32 / 4.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 180 gpurun_out/b6_drv1.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 180 gpurun_out/b6_drv2.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
for B in 128 32 4; do
  $S 240 gpurun_out/b6_prof$B.log rocprofv3 --kernel-trace -d gpurun_out/prof$B -o run -- python bench.py --steps 60 --warmup 4 --batch $B || exit 1
  python scripts/prof_timeline.py gpurun_out/prof$B/run_results.db > gpurun_out/timeline_b$B.txt 2>&1
done
echo ALLDONE
