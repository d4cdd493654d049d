# Runs the CPU test tier (what the driver runs without a GPU) on the GPU box.
set -o pipefail
mkdir -p gpurun_out
HIP_VISIBLE_DEVICES= timeout -k 10 900 python -u -m pytest tests -x -q -m "not gpu" -p no:cacheprovider --timeout 300 > gpurun_out/cpu_tier.log 2>&1
rc=$?; tail -3 gpurun_out/cpu_tier.log; exit $rc
