#!/bin/bash
# Two nodes, one on the CPU and one on the GPU, in one gloo-backed tree
# (reference: examples/client_remote.sh).  Set HOST to the root's address.
HOST=${HOST:-127.0.0.1}
PORT=${PORT:-8080}
cd "$(dirname "$0")/.."
OMP_NUM_THREADS=4 python examples/client_remote.py --nodeIndex 1 --numNodes 2 --host "$HOST" --port "$PORT" --backend gloo "$@" &
python examples/client_remote.py --nodeIndex 2 --numNodes 2 --host "$HOST" --port "$PORT" --backend gloo --cuda "$@"
wait
