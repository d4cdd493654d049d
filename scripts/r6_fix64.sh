#!/bin/bash
# 64x64-tile in-launch split-K combine (small-batch plans): kernel + executor
# tests, driver bench at batch 4 / 32 / 128, batch-4 sweep and timeline.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/f64_tests.log python -u -m pytest tests/kernels/test_convnet_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "fix or in_launch or matches_torch_model or fused_combine" || exit 1
for B in 4 32 128; do
  $S 200 gpurun_out/f64_b$B.log python bench.py --batch $B || exit 1
done
$S 300 gpurun_out/f64_sweep_b4.jsonl python scripts/sweep_small_batch.py --batch 4 || exit 1
$S 240 gpurun_out/f64_prof4.log rocprofv3 --kernel-trace -d gpurun_out/f64prof4 -o run -- python bench.py --steps 60 --warmup 4 --batch 4 || exit 1
python scripts/prof_timeline.py gpurun_out/f64prof4/run_results.db > gpurun_out/f64_timeline_b4.txt 2>&1
echo ALLDONE
