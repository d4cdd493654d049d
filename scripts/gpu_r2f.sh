#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/pytest_gpu.log python -u -m pytest tests/kernels/test_mnist_gpu.py tests/kernels/test_conv_resnet_gpu.py tests/kernels/test_resnet_gpu.py tests/kernels/test_engine_gpu.py -x -q -rs --timeout 150 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed\| error" gpurun_out/pytest_gpu.log || { echo "TESTS FAILED"; exit 1; }
$S 120 gpurun_out/bench_20.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 300 gpurun_out/bench_r50_hip.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
DISTLEARN_RESNET_FUSE_STATS=0 $S 300 gpurun_out/bench_r50_nofuse.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
$S 300 gpurun_out/diag_r50.log python scripts/diag_r50_graph.py || exit 1
$S 300 gpurun_out/bench_r50_graph.log python bench.py --model resnet50 --steps 20 --warmup 5 --graph 1 || exit 1
$S 200 gpurun_out/bench_mnist.log python scripts/bench_mnist.py --steps 2000 || exit 1
echo ALLDONE
