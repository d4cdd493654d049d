set -o pipefail
DISTLEARN_BENCH_TRACE=1 timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 20 --warmup 5 > gpurun_out/rn1.log 2>&1
grep "step" gpurun_out/rn1.log | tr '\n' ' '; echo
DISTLEARN_BENCH_TRACE=1 timeout -k 5 300 python bench.py --model resnet50 --steps 20 --warmup 5 > gpurun_out/rn2.log 2>&1
grep "step" gpurun_out/rn2.log | tr '\n' ' '; tail -1 gpurun_out/rn2.log | cut -c1-200
