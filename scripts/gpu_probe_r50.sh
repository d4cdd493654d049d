#!/bin/bash
# graph-branch concurrency probe + ResNet-50 bench and kernel profile
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python scripts/graph_branch_probe.py > gpurun_out/probe.txt 2>&1 || exit 1
cat gpurun_out/probe.txt
timeout -k 10 400 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/bench_r50.log 2>&1 || { tail -20 gpurun_out/bench_r50.log; exit 1; }
tail -1 gpurun_out/bench_r50.log
echo ALLDONE
