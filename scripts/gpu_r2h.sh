#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 gpurun_out/prof_mnist.log rocprofv3 --kernel-trace --stats -d gpurun_out/profm -o run -- python scripts/bench_mnist.py --steps 300 --only hip-graph || exit 1
python scripts/prof_summary.py gpurun_out/profm --steps 320 --top 15 > gpurun_out/kernels_mnist.txt 2>&1
$S 200 gpurun_out/prof_mnist_t.log rocprofv3 --kernel-trace --stats -d gpurun_out/profmt -o run -- python scripts/bench_mnist.py --steps 300 --only torch-graph || exit 1
python scripts/prof_summary.py gpurun_out/profmt --steps 320 --top 25 > gpurun_out/kernels_mnist_torch.txt 2>&1


$S 300 gpurun_out/bench_r50.log python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
DISTLEARN_MIOPEN_FIND=1 $S 400 gpurun_out/bench_r50_find.log python bench.py --model resnet50 --steps 20 --warmup 8 || exit 1
$S 300 gpurun_out/rocprof_r50.log rocprofv3 --kernel-trace --stats -d gpurun_out/prof50 -o run -- python bench.py --model resnet50 --steps 10 --warmup 3 || exit 1
python scripts/prof_summary.py gpurun_out/prof50 --steps 13 --top 45 > gpurun_out/kernels_r50.txt 2>&1
rm -rf gpurun_out/profm gpurun_out/profmt gpurun_out/prof50
echo ALLDONE
