set -o pipefail
for v in 0 1 0 1 0 1; do echo "# nosplit $v"; DISTLEARN_FWD_NOSPLIT=$v timeout -k 5 120 python bench.py --steps 600 --warmup 24 2>&1 | tail -1 | cut -c100-160 || exit 1; done
