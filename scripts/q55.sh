set -o pipefail
for st in 2 3; do for r in 0 1; do echo "# stages $st occupy $r"; timeout -k 5 180 python scripts/bench_conv.py --iters 100 --stages $st,0 --occupy $r 2>&1 | grep -E "^(fwd4|dgrad[34])" || exit 1; done; done
