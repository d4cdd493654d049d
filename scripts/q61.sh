set -o pipefail
timeout -k 5 400 python -u -m pytest tests/kernels -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
for v in 0 1 0 1 0 1; do echo "# fused $v"; DISTLEARN_HEAD_WGRAD_FUSED=$v timeout -k 5 120 python bench.py --steps 600 --warmup 24 2>&1 | tail -1 | cut -c100-160 || exit 1; done
