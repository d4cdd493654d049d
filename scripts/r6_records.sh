#!/bin/bash
# Round-6 records: full GPU suite, driver-form bench, AllReduceEA, world>1 path,
# ResNet-50 (checks the round-6 cleanup left it unchanged).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 900 gpurun_out/rec_tests.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
$S 200 gpurun_out/rec_drv.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 200 gpurun_out/rec_ea.log python bench.py --algo ea || exit 1
$S 200 gpurun_out/rec_nw.log python bench.py --nworld-path 1 || exit 1
$S 400 gpurun_out/rec_r50.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
echo ALLDONE
