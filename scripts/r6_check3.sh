#!/bin/bash
# bf16 delta-wire kernel tests, MNIST batch-1 re-measure, AsyncEA server model,
# CIFAR step timeline (batch 128) and PMC passes over the whole step.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/c3_tests.log python -u -m pytest tests/kernels/test_flat_ops_gpu.py tests/kernels/test_engine_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "elastic or async" || exit 1
$S 300 gpurun_out/c3_mnist_b1.log python scripts/bench_mnist.py --batch 1 || exit 1
$S 300 gpurun_out/c3_async_model.log python scripts/async_server_model.py --out gpurun_out/r6_async_server_model.json || exit 1
$S 240 gpurun_out/c3_prof128.log rocprofv3 --kernel-trace -d gpurun_out/c3prof128 -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/c3prof128/run_results.db > gpurun_out/c3_timeline_b128.txt 2>&1
PMC_CMD="python bench.py --steps 8 --warmup 2" timeout -k 10 500 bash scripts/pmc_hotpath.sh > gpurun_out/c3_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/c3_pmc.log; exit 1; }
echo ALLDONE
