#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/pytest_gpu.log python -u -m pytest tests/kernels/test_mnist_gpu.py tests/examples -m gpu -x -q -rs --timeout 150 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed\| error" gpurun_out/pytest_gpu.log || { echo "TESTS FAILED"; exit 1; }
$S 200 gpurun_out/bench_mnist.log python scripts/bench_mnist.py --steps 2000 || exit 1
$S 200 gpurun_out/bench_mnist16.log python scripts/bench_mnist.py --steps 1000 --batch 16 || exit 1
$S 200 gpurun_out/prof_mnist.log rocprofv3 --kernel-trace --stats -d gpurun_out/profm -o run -- python scripts/bench_mnist.py --steps 300 --only hip-graph || exit 1
python scripts/prof_summary.py gpurun_out/profm --steps 320 --top 12 > gpurun_out/kernels_mnist.txt 2>&1
rm -rf gpurun_out/profm
$S 300 gpurun_out/bench_r50.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
echo ALLDONE
