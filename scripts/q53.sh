set -o pipefail
E=scripts/emulate_rccl.py
timeout -k 5 180 python $E --cus 0,-1,1,-8,8,0 2>&1 | grep -E "occupied|Error" || exit 1
