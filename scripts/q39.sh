set -o pipefail
for it in 0 2 0 2; do
echo "# items $it"
DISTLEARN_BN_BWD_ITEMS=$it timeout -k 5 120 python bench.py --steps 400 --warmup 24 2>&1 | tail -1 | cut -c1-150 || exit 1
done
