#!/bin/bash
# AsyncEA: 1 server + N clients + 1 tester (reference: examples/AsyncEASGD.sh).
# Roles come from the rank: 0 = server, 1..N = clients, N+1 = tester.
# On a GPU node add --cuda (one GPU per role).
N=${N:-2}
cd "$(dirname "$0")/.." && python -m torch_distlearn_amd.launch --nproc $((N + 2)) --no-node-flags \
  examples/easgd.py --numNodes "$N" "$@"
