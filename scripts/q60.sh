set -o pipefail
export TMPDIR=/tmp
timeout -k 5 300 python -u -m pytest tests/kernels/test_flat_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
rm -rf gpurun_out/prof
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_summary.py gpurun_out/prof --steps 64 --top 40 > gpurun_out/kernels.txt 2>&1
grep -E "sgd|head|pool_fwd" gpurun_out/kernels.txt
