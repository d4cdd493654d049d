set -o pipefail
for wt in 0 2; do for st in 3 4; do for pf in 0 1; do
echo "# wtile $wt stages $st pf $pf"
timeout -k 5 120 python scripts/bench_conv.py --only wgrad --wtile $wt --stages 3,$st --wpf $pf --iters 100 2>&1 | grep "^wgrad[234]" || exit 1
done; done; done
