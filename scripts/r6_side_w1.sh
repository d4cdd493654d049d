#!/bin/bash
# Block 2's SGD update as extra workgroups of the first layer's weight-gradient
# launch (DISTLEARN_SIDE_WGRAD1=1) vs in the final update launch (=0).
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_engine_gpu.py \
  -k "deferred_slab_reduce or side or prep_next" > gpurun_out/sidew_tests.log 2>&1 || { tail -30 gpurun_out/sidew_tests.log; exit 1; }
tail -2 gpurun_out/sidew_tests.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/kernels/test_convnet_gpu.py \
  -k "executor" > gpurun_out/sidew_tests2.log 2>&1 || { tail -30 gpurun_out/sidew_tests2.log; exit 1; }
tail -2 gpurun_out/sidew_tests2.log
for v in 1 0; do
  DISTLEARN_SIDE_WGRAD1=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sidew_prof$v -o run -- python bench.py --steps 20 --warmup 5 \
    > gpurun_out/sidew_prof.log 2>&1 || { tail -20 gpurun_out/sidew_prof.log; exit 1; }
done
: > gpurun_out/sidew_ab.txt
for r in 1 2 3 4 5; do
  for v in 1 0 0 1; do
    DISTLEARN_SIDE_WGRAD1=$v timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/sidew_run.log 2>&1 || { tail -5 gpurun_out/sidew_run.log; exit 1; }
    echo "side_wgrad1=$v round=$r $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/sidew_run.log)" | tee -a gpurun_out/sidew_ab.txt
  done
done
echo ALLDONE
