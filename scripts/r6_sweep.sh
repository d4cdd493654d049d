set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
for B in 4 32 128; do
  $S 300 gpurun_out/sweep_b$B.jsonl python scripts/sweep_small_batch.py --batch $B || exit 1
done
echo ALLDONE
