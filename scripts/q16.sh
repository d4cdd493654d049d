set -o pipefail
timeout -k 5 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit 1
DISTLEARN_RCCL_WORLD1=1 timeout -k 5 120 python bench.py --steps 400 --warmup 24 > gpurun_out/bench_rccl1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_rccl1.log | cut -c1-150
