set -o pipefail
E=scripts/emulate_rccl.py
echo "# default"; timeout -k 5 180 python $E --cus 0,8,32 2>&1 | grep -E "occupied|Error" || exit 1
echo "# tile2 st4 nopf"; DISTLEARN_WGRAD_PF=0 DISTLEARN_WGRAD_STAGES=4 timeout -k 5 180 python $E --cus 0,8,32 2>&1 | grep -E "occupied|Error" || exit 1
echo "# tile0 st3 nopf"; DISTLEARN_WGRAD_TILE=0 timeout -k 5 180 python $E --cus 0,8,32 2>&1 | grep -E "occupied|Error" || exit 1
echo "# tile0 st4 pf"; DISTLEARN_WGRAD_TILE=0 DISTLEARN_WGRAD_STAGES=4 timeout -k 5 180 python $E --cus 0,8,32 2>&1 | grep -E "occupied|Error" || exit 1
echo "# region off"; DISTLEARN_REGION=0 timeout -k 5 180 python $E --cus 0,8,32 2>&1 | grep -E "occupied|Error" || exit 1
