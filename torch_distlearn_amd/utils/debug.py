"""Divergence detection for data-parallel replicas (SURVEY §5.2 "race
detection": the reference has none beyond handshake-string asserts).

:func:`assert_replicas_in_sync` all-reduces a float64 checksum of the flat
parameter buffer (sum and sum of |x|, plus min/max over ranks) and raises if
the replicas disagree -- the cheap end-to-end check that the collective
sequence, the uneven-step drain and the RCCL reductions kept every node
bitwise identical.  ``DISTLEARN_DEBUG_SYNC=1`` makes
``AllReduceSGD.synchronizeParameters`` run it automatically.

:func:`check_collective_sequence` (also under ``DISTLEARN_DEBUG_SYNC=1``)
compares the hash of every rank's issued collective sequence
(``Communicator.seq_state``, graph replays included) at the algorithms' epoch
synchronisation, after the drain -- RCCL hangs or silently mixes buffers when
ranks issue different sequences; this turns that into a ``CommError`` naming
the ranks.
"""
from __future__ import annotations

import os

import torch


def params_checksum(buf: torch.Tensor) -> torch.Tensor:
    b = buf.detach().double()
    return torch.stack([b.sum(), b.abs().sum(), (b * torch.arange(1, b.numel() + 1, device=b.device,
                                                                  dtype=torch.float64) % 1021).sum()]).cpu()


def assert_replicas_in_sync(tree, buf: torch.Tensor, what: str = "parameters") -> None:
    c = params_checksum(buf)
    hi, lo = c.clone(), c.clone()
    tree.comm.all_reduce_host(hi, "max")
    tree.comm.all_reduce_host(lo, "min")
    if not torch.equal(hi, lo):
        raise RuntimeError(f"replica divergence detected in {what} on node {tree.nodeIndex}: "
                           f"checksum range {lo.tolist()} .. {hi.tolist()}")


def debug_sync_enabled() -> bool:
    return os.environ.get("DISTLEARN_DEBUG_SYNC", "0") == "1"


def check_collective_sequence(tree, what: str) -> None:
    """Raise :class:`~torch_distlearn_amd.parallel.comm.CommError` when the
    ranks' collective sequences (op, dtype, count, op / root of every
    collective issued so far) differ.  Collective (control plane); a no-op
    unless ``DISTLEARN_DEBUG_SYNC=1``."""
    from ..parallel.comm import CommError, seq_tracking

    comm = tree.comm
    if comm.world_size <= 1 or not seq_tracking():
        return
    h, n = comm.seq_state()
    mine = torch.tensor([h >> 32, h & 0xFFFFFFFF, n], dtype=torch.int64)
    every = [tuple(int(v) for v in t.tolist()) for t in comm.all_gather_host(mine)]
    if len(set(every)) == 1:
        return
    groups = {}
    for r, v in enumerate(every):
        groups.setdefault(v, []).append(r + 1)
    desc = "; ".join(f"nodes {nodes}: {v[2]} collectives, hash {(v[0] << 32) | v[1]:016x}"
                     for v, nodes in sorted(groups.items(), key=lambda kv: kv[1]))
    raise CommError(f"collective sequence diverged before {what} (seen on node {tree.nodeIndex}): {desc}")
