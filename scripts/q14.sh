set -o pipefail
export NCCL_DEBUG=WARN
timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 40 --warmup 8 > gpurun_out/bench2.log 2>&1
echo "rc=$?"; tail -30 gpurun_out/bench2.log
