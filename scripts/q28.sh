set -o pipefail
DISTLEARN_BENCH_TRACE=1 timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 8 --warmup 5 > gpurun_out/rn2.log 2>&1
echo "plain: $(grep '^step' gpurun_out/rn2.log | tr '\n' ' ')"
DISTLEARN_DBG_SYNC_CAPTURE=1 DISTLEARN_BENCH_TRACE=1 timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 8 --warmup 5 > gpurun_out/rn3.log 2>&1
echo "sync-capture: $(grep '^step' gpurun_out/rn3.log | tr '\n' ' ')"
DISTLEARN_BENCH_TRACE=1 timeout -k 5 300 python bench.py --model resnet50 --batch 64 --steps 8 --warmup 6 > gpurun_out/rn4.log 2>&1
echo "warmup6: $(grep '^step' gpurun_out/rn4.log | tr '\n' ' ')"
