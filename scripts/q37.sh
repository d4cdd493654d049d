set -o pipefail
for st in 3 4; do
echo "# fwd stages $st"
timeout -k 5 120 python scripts/bench_conv.py --stages $st,0 --iters 100 2>&1 | grep -E "^(fwd|dgrad)[234]" || exit 1
done
