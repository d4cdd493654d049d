set -o pipefail
rm -f gpurun_out/stamps.txt
for st in 3 4 5 0; do for L in 2 4; do timeout -k 5 60 python scripts/stamp_region.py $L fwd 0 $st >> gpurun_out/stamps.txt 2>&1 || exit 1; done; done
for st in 3 4; do timeout -k 5 120 python scripts/bench_conv.py --iters 100 --region 1 --rstages $st --only fwd > gpurun_out/bc_st$st.txt 2>&1 || exit 1; done
