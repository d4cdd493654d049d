#!/bin/bash
# slab wgrad for the 1x1 convs + residual fusion default: numerics, microbench, ResNet bench + profile
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/kernels/test_conv_resnet_gpu.py tests/kernels/test_resnet_gpu.py > gpurun_out/t_conv.log 2>&1 || { tail -30 gpurun_out/t_conv.log; exit 1; }
tail -2 gpurun_out/t_conv.log
timeout -k 10 240 python scripts/bench_gemm1x1.py > gpurun_out/gemm1x1.jsonl 2> gpurun_out/gemm1x1.err || exit 1
timeout -k 10 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_r50.json 2> gpurun_out/bench_r50.err || exit 1
cat gpurun_out/bench_r50.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50 -o r50 -- python bench.py --model resnet50 --steps 5 --warmup 3 > gpurun_out/prof_r50.log 2>&1 || exit 1
python scripts/prof_summary.py gpurun_out/prof_r50 --steps 8 --top 60 > gpurun_out/r50_kernels.txt 2>&1 || true
rm -rf gpurun_out/prof_r50
