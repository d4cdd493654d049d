set -o pipefail
run() { timeout -k 5 120 python scripts/bench_conv.py --iters 100 --only $1 --wsplits $2 > gpurun_out/bc.log 2>&1; rc=$?; [ $rc -ge 124 ] && exit 1; grep -E "^wgrad" gpurun_out/bc.log || echo "$1 $2 failed $(tail -1 gpurun_out/bc.log|cut -c1-80)"; }
for sp in 64 96 128; do run wgrad1 $sp; done
for sp in 16 19 20; do run wgrad2 $sp; done
for sp in 4 5; do run wgrad3 $sp; done
exit 0
