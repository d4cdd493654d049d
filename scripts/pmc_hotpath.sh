#!/bin/bash
# PMC counters (one rocprofv3 pass per counter set, kernel trace for durations)
# of the hot kernels driven by scripts/pmc_hotpath.py (or by $PMC_CMD, e.g.
# PMC_CMD="python bench.py --steps 8 --warmup 2" for the CIFAR step); summary -> gpurun_out/pmc_hotpath.txt
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD=${PMC_CMD:-python scripts/pmc_hotpath.py --iters 3}
i=0
for P in "FETCH_SIZE GRBM_GUI_ACTIVE" "WRITE_SIZE GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P -d gpurun_out/pmch_p$i -o run -- $CMD > gpurun_out/pmch_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmch_p$i.log; exit 1; }
done
python scripts/pmc_hotpath_summary.py gpurun_out/pmch_p1 gpurun_out/pmch_p2 gpurun_out/pmch_p3 > gpurun_out/pmc_hotpath.txt 2>&1
rm -rf gpurun_out/pmch_p1 gpurun_out/pmch_p2 gpurun_out/pmch_p3
cat gpurun_out/pmc_hotpath.txt
