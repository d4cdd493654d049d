#!/bin/bash
# ad-hoc GPU check: new kernel tests, fused-combine timelines
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/kernels/test_conv_ex_gpu.py tests/kernels/test_resnet_strided_gpu.py tests/kernels/test_convnet_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_new.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_new.log
[ $rc -ge 124 ] && exit 1
for F in 1 0; do
  DISTLEARN_FUSE_COMBINE=$F timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof$F -o run -- python bench.py --steps 60 --warmup 4 > gpurun_out/rocprof$F.log 2>&1 || { echo "rocprof $F failed"; tail -5 gpurun_out/rocprof$F.log; exit 1; }
  python scripts/prof_timeline.py gpurun_out/prof$F/run_results.db > gpurun_out/timeline$F.txt 2>&1
  rm -rf gpurun_out/prof$F
  echo "== fuse $F"; grep -E "combine|reduce_kernel|span" gpurun_out/timeline$F.txt
done
echo ALLDONE
