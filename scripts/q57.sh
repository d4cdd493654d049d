set -o pipefail
E=scripts/emulate_rccl.py
echo "# world-1 config"; timeout -k 5 180 python $E --cus 0,16,32 2>&1 | grep -E "occupied|Error" || exit 1
echo "# overlap config (reserve 32, dgrad 2 stages)"; DISTLEARN_CU_RESERVE=32 DISTLEARN_DGRAD_STAGES=2 timeout -k 5 180 python $E --cus 0,16,32 2>&1 | grep -E "occupied|Error" || exit 1
