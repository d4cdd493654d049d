set -o pipefail
for L in 2 3 4; do for m in fwd dgrad; do timeout -k 5 60 python scripts/stamp_region.py $L $m >> gpurun_out/stamps.txt 2>&1 || exit 1; done; done
