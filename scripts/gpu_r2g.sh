#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 gpurun_out/bench_mnist.log python scripts/bench_mnist.py --steps 2000 || exit 1
$S 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -rs --timeout 150 --timeout-method thread || exit 1
grep -q " passed" gpurun_out/pytest_gpu.log && ! grep -q " failed\| error" gpurun_out/pytest_gpu.log || { echo "TESTS FAILED"; exit 1; }
$S 180 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 120 gpurun_out/bench_20.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 300 gpurun_out/bench_r50.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
echo ALLDONE
