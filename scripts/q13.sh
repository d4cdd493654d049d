set -o pipefail
C=tests/kernels/test_convnet_gpu.py
timeout -k 5 300 python -u -m pytest $C -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/t_conv.log 2>&1; rc=$?; tail -2 gpurun_out/t_conv.log
[ $rc -ne 0 ] && exit 1
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --only wgrad > gpurun_out/bc_wg.txt 2>&1 || exit 1
