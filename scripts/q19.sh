set -o pipefail
timeout -k 5 300 python scripts/debug_resnet.py --graph 1 --batch 256 --steps 26 --bucket-mb 16 > gpurun_out/dbg_r3.txt 2>&1
timeout -k 5 300 python scripts/debug_resnet.py --graph 0 --batch 256 --steps 26 --bucket-mb 16 --port 29705 > gpurun_out/dbg_r4.txt 2>&1
