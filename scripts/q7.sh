set -o pipefail
rm -f gpurun_out/stamps.txt
for ab in 0 1 2 3; do timeout -k 5 60 python scripts/stamp_region.py 2 fwd $ab >> gpurun_out/stamps.txt 2>&1 || exit 1; done
for ab in 0 1 2 3; do timeout -k 5 60 python scripts/stamp_region.py 4 fwd $ab >> gpurun_out/stamps.txt 2>&1 || exit 1; done
