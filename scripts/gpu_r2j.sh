#!/bin/bash
# transposed-accumulator streaming conv kernel: numerics, 1x1 microbench, CIFAR + ResNet bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_convnet_gpu.py tests/kernels/test_conv_resnet_gpu.py > gpurun_out/t_conv.log 2>&1 || { tail -30 gpurun_out/t_conv.log; exit 1; }
tail -2 gpurun_out/t_conv.log
timeout -k 10 240 python scripts/bench_gemm1x1.py > gpurun_out/gemm1x1.jsonl 2> gpurun_out/gemm1x1.err || exit 1
timeout -k 10 200 python bench.py > gpurun_out/bench_cifar.json 2> gpurun_out/bench_cifar.err || exit 1
cat gpurun_out/bench_cifar.json
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.err || exit 1
cat gpurun_out/bench_r50.json
