set -o pipefail
timeout -k 5 400 python -u -m pytest tests/kernels -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; rc=$?; tail -1 gpurun_out/t.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/t.log | head -20; exit 1; }
HIP_VISIBLE_DEVICES= timeout -k 10 900 python -u -m pytest tests -x -q -m "not gpu" -p no:cacheprovider --timeout 300 > gpurun_out/cpu_tier.log 2>&1; rc=$?; tail -1 gpurun_out/cpu_tier.log; exit $rc
