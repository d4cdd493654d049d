#!/bin/bash
# Final round-6 records after the pair-packed layer 1: full GPU suite, smoke,
# driver-form bench, batches 32 / 4, EA, world>1 path, the comm-holding run.
set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
S=scripts/gpu_step.sh
$S 900 gpurun_out/fin_tests.log python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
$S 200 gpurun_out/fin_smoke.log python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" || exit 1
$S 200 gpurun_out/fin_drv.log python bench.py --gpus 1 --steps 20 --warmup 5 || exit 1
$S 200 gpurun_out/fin_drv50.log python bench.py || exit 1
$S 200 gpurun_out/fin_b32.log python bench.py --batch 32 || exit 1
$S 200 gpurun_out/fin_b4.log python bench.py --batch 4 || exit 1
$S 200 gpurun_out/fin_ea.log python bench.py --algo ea || exit 1
$S 200 gpurun_out/fin_nw.log python bench.py --nworld-path 1 || exit 1
$S 200 gpurun_out/fin_hold.log python bench.py --hold-cus 32 || exit 1
echo ALLDONE
