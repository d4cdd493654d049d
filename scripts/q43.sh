set -o pipefail
for L in dgrad3 dgrad4; do for t in 0 1 2; do for sp in 1 2 4 8; do
timeout -k 5 120 python scripts/bench_conv.py --only $L --dtile $t --dsplits $sp --iters 100 > gpurun_out/bc.log 2>&1; rc=$?
[ $rc -ge 124 ] && { echo "fatal rc=$rc"; exit 1; }
grep -E "^(fwd|dgrad)[34]" gpurun_out/bc.log || echo "$L tile$t split$sp failed: $(tail -1 gpurun_out/bc.log | cut -c1-100)"
done; done; done
exit 0
