set -o pipefail
timeout -k 5 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
grep -o "SQ_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|TA_[A-Z_0-9]*\|TCC_[A-Z_0-9]*" gpurun_out/counters_list.txt | sort -u > gpurun_out/counters_names.txt
echo done
