set -o pipefail
for args in "--batch 64" "--batch 64 --graph 0" "--batch 256 --graph 0"; do
timeout -k 5 300 python bench.py --model resnet50 --steps 20 --warmup 5 $args > gpurun_out/rn.log 2>&1 || exit 1
echo "$args: $(tail -1 gpurun_out/rn.log | grep -o '"ms_per_step": [0-9.]*\|"final_loss": [0-9.NaN]*' | tr '\n' ' ')"
done
