set -o pipefail
DISTLEARN_BENCH_TRACE=1 timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 20 --warmup 5 > gpurun_out/rn1.log 2>&1
grep "step\|final" gpurun_out/rn1.log | cut -c1-100 | tail -22
DISTLEARN_BENCH_TRACE=sync timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 20 --warmup 5 > gpurun_out/rn2.log 2>&1
grep "step" gpurun_out/rn2.log | tail -21 | tr '\n' ' '
