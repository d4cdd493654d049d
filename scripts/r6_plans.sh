#!/bin/bash
# Batch-aware plans: targeted GPU tests, driver-form bench
# at batch 128 / 32 / 4 and one-step kernel timelines at each batch.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/plans_tests.log python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "matches_torch_model or comm_profile or in_launch or fused_combine or dgrad_bn_reduce or device_loader or resume or unrolled or graph" || exit 1
for B in 128 32 4; do
  $S 200 gpurun_out/plans_b$B.log python bench.py --batch $B || exit 1
done
for B in 128 32 4; do
  $S 240 gpurun_out/plans_prof$B.log rocprofv3 --kernel-trace -d gpurun_out/pprof$B -o run -- python bench.py --steps 60 --warmup 4 --batch $B || exit 1
  python scripts/prof_timeline.py gpurun_out/pprof$B/run_results.db > gpurun_out/ptimeline_b$B.txt 2>&1
done
echo ALLDONE
