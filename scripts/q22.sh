set -o pipefail
timeout -k 5 300 python scripts/debug_resnet.py --graph 1 --batch 64 --steps 10 --sync 0 > gpurun_out/dbg_ns.txt 2>&1
tail -12 gpurun_out/dbg_ns.txt
