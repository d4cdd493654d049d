set -o pipefail
timeout -k 5 120 python scripts/bench_prep.py > gpurun_out/prep.txt 2>&1 && bash scripts/gpu_quick.sh "convnet or engine or gather or prep"
