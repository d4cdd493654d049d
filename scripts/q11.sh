set -o pipefail
export TMPDIR=/tmp
for r in 1 0; do
timeout -k 5 120 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_r$r -o run -- python scripts/bench_conv.py --iters 20 --region $r > gpurun_out/kt_r$r.log 2>&1 || exit 1
python scripts/prof_summary.py gpurun_out/kt_r$r --top 20 > gpurun_out/kt_r$r.txt
done
