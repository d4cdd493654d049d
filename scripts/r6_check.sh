set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 900 gpurun_out/gpu_tests.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
$S 300 gpurun_out/bench_b128.log python bench.py || exit 1
for B in 4 32; do
  $S 200 gpurun_out/bench_b$B.log python bench.py --batch $B || exit 1
done
for B in 4 32 128; do
  $S 300 gpurun_out/sweep_b$B.jsonl python scripts/sweep_small_batch.py --batch $B || exit 1
done
echo ALLDONE
