set -o pipefail
for wt in 0 2; do timeout -k 5 120 python scripts/bench_conv.py --only wgrad --wtile $wt --iters 100 2>&1 | grep -v "^#" || exit 1; done
timeout -k 5 120 python scripts/bench_conv.py --only wgrad --wtile 2 --stages 3,4 --iters 100 2>&1 | grep -v "^#"
