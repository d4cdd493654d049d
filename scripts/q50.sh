set -o pipefail
for v in 0 1; do echo "# pow2 $v"; DISTLEARN_WGRAD_POW2=$v timeout -k 5 180 python scripts/emulate_rccl.py --cus 0,8,16,32,56,64 --steps 400 2>&1 | grep -E "occupied|Error|error" || exit 1; done
