#!/bin/bash
# PMC counters of the fwd/dgrad conv kernels (region vs streaming), one pass per counter set.
#   usage: pmc_conv.sh <only-filter>   e.g. fwd2
set -o pipefail
export TMPDIR=/tmp
F=${1:-fwd2}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
for r in 1 0; do
  i=0
  for P in "$P1" "$P2"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_${F}_r${r}_p$i -o run -- python scripts/bench_conv.py --iters 5 --region $r --only $F > gpurun_out/pmc_${F}_r${r}_p$i.log 2>&1 || exit 1
  done
done
for r in 1 0; do for i in 1 2; do echo "== region=$r pass $i"; python scripts/pmc_summary.py gpurun_out/pmc_${F}_r${r}_p$i conv_fwd; done; done > gpurun_out/pmc_${F}.txt
