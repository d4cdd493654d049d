set -o pipefail
mkdir -p gpurun_out
timeout -k 5 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd or dgrad" > gpurun_out/t_conv.log 2>&1; rc=$?; tail -3 gpurun_out/t_conv.log
[ $rc -ne 0 ] && exit 1
for st in 0 3 4 6; do
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --region 1 --rstages $st --only d > gpurun_out/bc_st$st.txt 2>&1 || exit 1
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --region 1 --rstages $st --only fwd >> gpurun_out/bc_st$st.txt 2>&1 || exit 1
done
