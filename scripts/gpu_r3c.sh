#!/bin/bash
# Full GPU test suite, prep transpose taps-per-block A/B, ResNet-50 bench with the border-only zero fill, copy-kernel call sites.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 600 gpurun_out/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for t in 1 4; do
    DISTLEARN_PREP_TAPS=$t $S 120 gpurun_out/prep_t${t}_$rep.log python bench.py --steps 400 --warmup 24 || exit 1
  done
done
$S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
$S 300 gpurun_out/r50_1.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
$S 300 gpurun_out/r50_2.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
$S 300 gpurun_out/copies.log python scripts/diag_r50_copies.py || exit 1
$S 400 gpurun_out/rocprof_r50.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof50 -o run -- python bench.py --model resnet50 --steps 12 --warmup 5 || exit 1
python scripts/prof_summary.py gpurun_out/prof50 --steps 17 --top 60 > gpurun_out/r50_kernels.txt 2>&1
for f in gpurun_out/prep_t*.log gpurun_out/r50_?.log; do
  echo "$f $(grep -h '"metric"' $f | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
echo ALLDONE
