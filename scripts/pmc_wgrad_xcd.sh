#!/bin/bash
# L2 (TCC) hit rate of the weight-gradient kernels: 2-D grid (DISTLEARN_WGRAD_XCD=0)
# vs the split-major XCD-aware 1-D grid (1), on the headline bench step.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for X in 0 1; do
  DISTLEARN_WGRAD_XCD=$X timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_x$X -o run -- python bench.py --steps 20 --warmup 4 > gpurun_out/pmc_x$X.log 2>&1 || exit 1
  echo "== DISTLEARN_WGRAD_XCD=$X" >> gpurun_out/pmc_wgrad_xcd.txt
  python scripts/pmc_summary.py gpurun_out/pmc_x$X conv_wgrad >> gpurun_out/pmc_wgrad_xcd.txt
  rm -rf gpurun_out/pmc_x$X
done
cat gpurun_out/pmc_wgrad_xcd.txt
echo ALLDONE
