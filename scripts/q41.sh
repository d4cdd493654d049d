set -o pipefail
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof.log 2>&1 || exit 1
python scripts/prof_timeline.py gpurun_out/prof/run_results.db > gpurun_out/timeline.txt 2>&1
