#!/bin/bash
# Full GPU check on the gpurun box: GPU tests, smoke(), 1-GPU bench (sgd, ea,
# resnet50), rocprofv3 kernel stats + one-step timeline of the headline bench.
# Each step has its own time limit; a fault/timeout stops the script
# (scripts/gpu_step.sh).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
$S 180 gpurun_out/smoke.log python -c "import __graft_entry__ as g; g.smoke()" || exit 1
$S 180 gpurun_out/bench_driver.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 180 gpurun_out/bench_sgd.log python bench.py --steps 400 --warmup 24 || exit 1
$S 180 gpurun_out/bench_ea.log python bench.py --algo ea --steps 400 --warmup 24 || exit 1
$S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
python scripts/prof_summary.py gpurun_out/prof --steps 64 --top 40 > gpurun_out/kernels.txt 2>&1
$S 400 gpurun_out/bench_resnet50.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
echo ALLDONE
