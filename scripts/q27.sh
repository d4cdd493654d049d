set -o pipefail
DISTLEARN_BENCH_TRACE=sync timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 4 --warmup 5 > gpurun_out/rn2.log 2>&1
grep "step\|warmup" gpurun_out/rn2.log | grep -v "^{" 
DISTLEARN_BENCH_TRACE=sync timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 4 --warmup 5 --graph 0 > gpurun_out/rn3.log 2>&1
grep "step\|warmup" gpurun_out/rn3.log | grep -v "^{"
