#!/bin/bash
# dgrad weight transposes in the head launch (DISTLEARN_HEAD_TRANSPOSES 1) vs in prep (0):
# CIFAR kernel/engine tests, interleaved bench A/B, one-step timeline.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/pytest_cifar.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2; do
  for t in 0 1; do
    DISTLEARN_HEAD_TRANSPOSES=$t $S 120 gpurun_out/htr${t}_$rep.log python bench.py --steps 400 --warmup 24 || exit 1
  done
done
$S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
for f in gpurun_out/htr*.log; do
  echo "$f $(grep -h '"metric"' $f | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
echo ALLDONE
