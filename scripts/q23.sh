set -o pipefail
timeout -k 5 300 python scripts/debug_resnet.py --graph 1 --batch 64 --steps 6 --sync 0 --sync-params 1 > gpurun_out/dbg_sp.txt 2>&1
tail -6 gpurun_out/dbg_sp.txt
timeout -k 5 300 python scripts/debug_resnet.py --graph 0 --batch 64 --steps 6 --sync 0 --sync-params 1 --port 29709 > gpurun_out/dbg_sp0.txt 2>&1
tail -6 gpurun_out/dbg_sp0.txt
