#!/bin/bash
# PMC counters of the wgrad kernel for one layer, one pass per counter set.
#   usage: pmc_wgrad.sh <only-filter> [wtile]   e.g. wgrad4 0
set -o pipefail
export TMPDIR=/tmp
F=${1:-wgrad4}; WT=${2:--1}
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_ACTIVE_INST_LDS"
P3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_TA_BUSY_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc_${F}_p$i -o run -- python scripts/bench_conv.py --iters 5 --wtile $WT --only $F > gpurun_out/pmc_${F}_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${F}_p$i.log; }
done
for i in 1 2 3; do echo "== pass $i"; python scripts/pmc_summary.py gpurun_out/pmc_${F}_p$i conv_wgrad; done > gpurun_out/pmc_${F}.txt
cat gpurun_out/pmc_${F}.txt
