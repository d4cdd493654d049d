set -o pipefail
E=scripts/emulate_rccl.py
for st in 3 2; do echo "# dgrad stages $st"; DISTLEARN_DGRAD_STAGES=$st timeout -k 5 180 python $E --cus 0,8,32 2>&1 | grep -E "occupied|Error" || exit 1; done
