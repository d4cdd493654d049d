set -o pipefail
C=tests/kernels/test_convnet_gpu.py
timeout -k 5 300 python -u -m pytest $C -x -q --timeout 120 --timeout-method thread > gpurun_out/t_conv.log 2>&1; rc=$?; tail -2 gpurun_out/t_conv.log
[ $rc -ne 0 ] && exit 1
for st in "3,3" "3,4"; do timeout -k 5 120 python scripts/bench_conv.py --iters 100 --stages $st --only wgrad > gpurun_out/bc_wg$st.txt 2>&1 || exit 1; done
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --stages 3,3 --only wgrad --wtile 2 > gpurun_out/bc_wgt2.txt 2>&1 || exit 1
