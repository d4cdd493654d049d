set -o pipefail
timeout -k 5 300 python -u -m pytest tests/kernels/test_convnet_gpu.py -x -q --timeout 120 --timeout-method thread -k "fwd or dgrad" > gpurun_out/t_conv.log 2>&1; rc=$?; tail -3 gpurun_out/t_conv.log
[ $rc -ne 0 ] && exit 1
rm -f gpurun_out/stamps.txt
for L in 2 4; do timeout -k 5 60 python scripts/stamp_region.py $L fwd 0 >> gpurun_out/stamps.txt 2>&1 || exit 1; done
timeout -k 5 120 python scripts/bench_conv.py --iters 100 --region 1 > gpurun_out/bc_r1.txt 2>&1 || exit 1
