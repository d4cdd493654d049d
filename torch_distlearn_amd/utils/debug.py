"""Divergence detection for data-parallel replicas (SURVEY §5.2 "race
detection": the reference has none beyond handshake-string asserts).

:func:`assert_replicas_in_sync` all-reduces a float64 checksum of the flat
parameter buffer (sum and sum of |x|, plus min/max over ranks) and raises if
the replicas disagree -- the cheap end-to-end check that the collective
sequence, the uneven-step drain and the RCCL reductions kept every node
bitwise identical.  ``DISTLEARN_DEBUG_SYNC=1`` makes
``AllReduceSGD.synchronizeParameters`` run it automatically.
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
