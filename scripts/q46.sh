set -o pipefail
for w in 8 4; do echo "# waves $w"; timeout -k 5 120 python scripts/bench_conv.py --waves $w --iters 100 2>&1 | grep -E "^(fwd|dgrad)[234]" || exit 1; done
