#!/bin/bash
# Engine GPU tests (timestamp calibration, replay profile) and the world>1 step timeline.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 300 gpurun_out/nw_tests.log python -u -m pytest tests/kernels/test_engine_gpu.py tests/kernels/test_mnist_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
$S 240 gpurun_out/nw_prof.log rocprofv3 --kernel-trace -d gpurun_out/nwprof -o run -- python bench.py --nworld-path 1 --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/nwprof/run_results.db > gpurun_out/nw_timeline.txt 2>&1
$S 240 gpurun_out/n1_prof.log rocprofv3 --kernel-trace -d gpurun_out/n1prof -o run -- python bench.py --steps 60 --warmup 4 || exit 1
python scripts/prof_timeline.py gpurun_out/n1prof/run_results.db > gpurun_out/n1_timeline.txt 2>&1
echo ALLDONE
