#!/bin/bash
# Engine GPU tests (replay comm profile, device-loader ring), the fused
# combine at 16 splits, driver bench at batch 128 / 32 / 4, world>1 path.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/c2_tests.log python -u -m pytest tests/kernels/test_engine_gpu.py tests/kernels/test_convnet_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "engine_gpu or fused_combine or matches_torch_model" || exit 1
for B in 128 32 4; do
  $S 200 gpurun_out/c2_b$B.log python bench.py --batch $B || exit 1
done
$S 200 gpurun_out/c2_nw.log python bench.py --nworld-path 1 || exit 1
$S 240 gpurun_out/c2_prof4.log rocprofv3 --kernel-trace -d gpurun_out/c2prof4 -o run -- python bench.py --steps 60 --warmup 4 --batch 4 || exit 1
python scripts/prof_timeline.py gpurun_out/c2prof4/run_results.db > gpurun_out/c2_timeline_b4.txt 2>&1
$S 300 gpurun_out/c2_async_model.log python scripts/async_server_model.py --out gpurun_out/r6_async_server_model.json || exit 1
echo ALLDONE
