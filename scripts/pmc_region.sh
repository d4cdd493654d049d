#!/bin/bash
# LDS counters of the region kernel (layer 2 fwd), plain and ablated (3 = no DMA, no MFMA)
set -o pipefail
export TMPDIR=/tmp
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAIT_INST_LDS"
for ab in 0 3; do
  timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmcr_$ab -o run -- python scripts/stamp_region.py 2 fwd $ab > gpurun_out/pmcr_$ab.log 2>&1 || exit 1
  echo "== ablate $ab" >> gpurun_out/pmc_region.txt
  python scripts/pmc_summary.py gpurun_out/pmcr_$ab region >> gpurun_out/pmc_region.txt
done
