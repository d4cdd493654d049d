#!/bin/bash
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/c4_tests.log python -u -m pytest tests/kernels/test_convnet_gpu.py tests/kernels/test_engine_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "executor or fix or engine_gpu" || exit 1
$S 200 gpurun_out/c4_b128.log python bench.py || exit 1
$S 200 gpurun_out/c4_drv.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 200 gpurun_out/c4_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" || exit 1
echo ALLDONE
