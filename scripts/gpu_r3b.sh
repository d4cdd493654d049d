#!/bin/bash
# Round-3 A/B: per-bucket SGD on the comm stream (DISTLEARN_BUCKET_UPDATE 0/1),
# BN apply rows (DISTLEARN_BN_TUNE 2,256 vs default 4,256), engine GPU tests,
# one-step timeline with the per-bucket update.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 400 gpurun_out/pytest_eng.log python -u -m pytest tests/kernels/test_engine_gpu.py tests/kernels/test_multirank_gpu.py tests/kernels/test_rccl_multigpu.py tests/kernels/test_convnet_gpu.py -x -q --timeout 200 --timeout-method thread || exit 1
for rep in 1 2 3; do
  for u in 0 1; do
    DISTLEARN_BUCKET_UPDATE=$u $S 120 gpurun_out/sgd_u${u}_$rep.log python bench.py --steps 20 --warmup 5 || exit 1
    DISTLEARN_BUCKET_UPDATE=$u $S 120 gpurun_out/sgd400_u${u}_$rep.log python bench.py --steps 400 --warmup 24 || exit 1
  done
done
$S 240 gpurun_out/rocprof.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
for rep in 1 2; do
  for t in 2,256 4,256; do
    DISTLEARN_BN_TUNE=$t $S 300 gpurun_out/r50_${t}_$rep.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
  done
done
for f in gpurun_out/sgd*_u*.log gpurun_out/r50_*.log; do
  echo "$f $(grep -h '"metric"' $f | python -c "import sys,json; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
echo ALLDONE
