#!/bin/bash
# MFMA work of the layer-4 forward / dgrad with pixel-major (DISTLEARN_POSM=0) vs
# position-major tiles that skip the zero-border taps (1)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for X in 0 1; do
  DISTLEARN_POSM=$X timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_p$X -o run -- python bench.py --steps 20 --warmup 4 > gpurun_out/pmc_p$X.log 2>&1 || exit 1
  echo "== DISTLEARN_POSM=$X" >> gpurun_out/pmc_posm.txt
  python scripts/pmc_summary.py gpurun_out/pmc_p$X "conv_fwd_kernel<128, 128, false, true" >> gpurun_out/pmc_posm.txt
  rm -rf gpurun_out/pmc_p$X
done
cat gpurun_out/pmc_posm.txt
echo ALLDONE
