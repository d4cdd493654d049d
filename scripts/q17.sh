set -o pipefail
timeout -k 5 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "head" > gpurun_out/t_head.log 2>&1; rc=$?; tail -2 gpurun_out/t_head.log
[ $rc -ne 0 ] && exit 1
timeout -k 5 120 python scripts/bench_prep.py > gpurun_out/prep.txt 2>&1 || exit 1
