#!/bin/bash
# GPU tests (incl. multi-GPU rows that skip on 1 GPU, watchdog), smoke, and the
# driver's bench command next to a 400-step run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 500 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q -rs --timeout 150 --timeout-method thread || exit 1
$S 180 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 120 gpurun_out/bench_20a.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 120 gpurun_out/bench_20b.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 180 gpurun_out/bench_400.log python bench.py --steps 400 --warmup 24 || exit 1
echo ALLDONE
