set -o pipefail
timeout -k 5 300 python scripts/debug_resnet.py --graph 0 --batch 64 --steps 6 --seed 1234 --lr 0.02 > gpurun_out/dbg_s0.txt 2>&1; grep step gpurun_out/dbg_s0.txt
timeout -k 5 300 python scripts/debug_resnet.py --graph 1 --batch 64 --steps 6 --seed 1234 --lr 0.02 --port 29710 > gpurun_out/dbg_s1.txt 2>&1; grep step gpurun_out/dbg_s1.txt
