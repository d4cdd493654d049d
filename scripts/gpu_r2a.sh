#!/bin/bash
# Round-2 first GPU pass: GPU tests, the driver's exact bench command (twice),
# the 400-step bench for the 20-vs-400 consistency check, and the EA bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
$S 120 gpurun_out/bench_20a.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 120 gpurun_out/bench_20b.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 180 gpurun_out/bench_400.log python bench.py --steps 400 --warmup 24 || exit 1
$S 180 gpurun_out/bench_ea.log python bench.py --algo ea --steps 400 --warmup 24 || exit 1
echo ALLDONE
