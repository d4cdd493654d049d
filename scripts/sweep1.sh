set -o pipefail
mkdir -p gpurun_out
for cfg in "--waves 8" "--waves 4" "--waves 4 --wtile 2" "--waves 8 --wtile 2" "--waves 4 --stages 3,4" "--waves 4 --wtile 2 --stages 3,2" "--waves 4 --stages 4,3"; do
  echo "=== $cfg" >> gpurun_out/sweep1.txt
  timeout -k 5 120 python scripts/bench_conv.py --iters 100 $cfg >> gpurun_out/sweep1.txt 2>&1 || exit 1
done
