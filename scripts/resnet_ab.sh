#!/bin/bash
# ResNet-50 (BASELINE config 5): BatchNorm precision A/B back to back on one
# box, BN numerics check, hipGraph attempt; data-plane bandwidth sweep.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 200 gpurun_out/r50_bn_check.log python scripts/resnet_bn_check.py || exit 1
$S 200 gpurun_out/r50_bn_fp32.log env DISTLEARN_RESNET_BN=fp32 python bench.py --model resnet50 --steps 20 --warmup 5 || exit 1
$S 200 gpurun_out/r50_bn_mixed.log env DISTLEARN_RESNET_BN=mixed python bench.py --model resnet50 --steps 40 --warmup 5 || exit 1
$S 200 gpurun_out/r50_bn_mixed_graph.log env DISTLEARN_RESNET_BN=mixed python bench.py --model resnet50 --steps 40 --warmup 5 --graph 1 || exit 1
$S 200 gpurun_out/allreduce_bw_w1.log python scripts/allreduce_bw.py --max-mb 64 || exit 1
echo ALLDONE
