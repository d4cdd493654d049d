set -o pipefail
mkdir -p gpurun_out
timeout -k 5 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_conv.log 2>&1; rc=$?; tail -15 gpurun_out/t_conv.log
[ $rc -ge 124 ] && exit 1
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --region 1 > gpurun_out/bc_r1.txt 2>&1 || exit 1
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --region 0 > gpurun_out/bc_r0.txt 2>&1 || exit 1
exit $rc
