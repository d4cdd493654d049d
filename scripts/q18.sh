set -o pipefail
timeout -k 5 200 python scripts/debug_resnet.py --graph 0 --batch 64 --steps 8 > gpurun_out/dbg_r0.txt 2>&1
timeout -k 5 200 python scripts/debug_resnet.py --graph 1 --batch 64 --steps 8 --port 29702 > gpurun_out/dbg_r1.txt 2>&1
timeout -k 5 200 python scripts/debug_resnet.py --graph 0 --batch 64 --steps 8 --lr 0.01 --port 29703 > gpurun_out/dbg_r2.txt 2>&1
