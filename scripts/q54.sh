set -o pipefail
for r in 0 1; do echo "# occupy $r"; timeout -k 5 180 python scripts/bench_conv.py --iters 100 --occupy $r 2>&1 | grep -E "^(fwd|dgrad|wgrad)" || exit 1; done
