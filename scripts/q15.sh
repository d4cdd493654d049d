set -o pipefail
timeout -k 5 400 python -u -m pytest tests/kernels/test_multirank_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_mr.log 2>&1; rc=$?; tail -15 gpurun_out/t_mr.log; exit $rc
