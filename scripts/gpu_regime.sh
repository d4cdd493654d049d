#!/bin/bash
# The reference's regime: global batch 32 (examples/cifar10.lua:6,36) vs the bench's 128 per GPU;
# the example on the fast path vs bench.py at the same batch.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 32 128; do
  timeout -k 10 180 python bench.py --batch $B --steps 400 --warmup 24 > gpurun_out/bench_b$B.log 2>&1 || { tail -5 gpurun_out/bench_b$B.log; exit 1; }
  echo "bench batch $B: $(tail -1 gpurun_out/bench_b$B.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/step", d["value"], "img/s")')"
  timeout -k 10 300 python -m torch_distlearn_amd.launch --nproc 1 --gpus examples/cifar10.py --epochs 2 --batchSize $B --trainSize 50000 --testSize 1000 > gpurun_out/example_b$B.log 2>&1 || { tail -5 gpurun_out/example_b$B.log; exit 1; }
  grep "img/s" gpurun_out/example_b$B.log
done
echo ALLDONE
