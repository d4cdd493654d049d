"""``Tree`` / ``LocalhostTree``: the collective topology object the algorithms
are built on, with the reference's exact contract.

Reference: ``ipc.Tree(nodeIndex, numNodes, base, server, client, host, port)``
and ``ipc.LocalhostTree(nodeIndex, numNodes)`` (test/test_AllReduceSGD.lua:7,
examples/mnist.lua:16, examples/client_remote.lua:31-41) returning
``{nodeIndex, numNodes, walkTable, allReduce, scatter}``.

``allReduce(value, op[, zero]) -> (value, n)`` (inferred contract):

* **normal call** (``zero is None``): one collective round; the result is
  written in place into ``value``; ``n`` = number of nodes that made a normal
  call in this round.
* **drain call** (``zero`` given): repeat rounds; each round contributes
  ``zero(tensor_i, i)`` (1-based ``i``) for every leaf of ``value`` (or of the
  last reduced layout when ``value is None``), *not* counted in ``n``; the
  in-place result of round k is visible to round k+1's callback; stop after the
  first round with ``n == 0`` (everyone is draining).

MI355X implementation: the reference walks the table and ships every tensor
over TCP up and down a b-ary tree.  Here the leaves are packed into one flat
buffer per (device, dtype) with a 64-element header whose element 0 carries the
participation count (1 or 0), and that buffer is reduced by ONE RCCL
all-reduce per dtype (grouped), so ``n`` arrives with the data.  Values that
are already flat (:class:`FlatBuffer`, e.g. the persistent gradient buffer of
:class:`~torch_distlearn_amd.ops.flat.FlatParams`) are reduced zero-copy.
``base`` (tree arity) is accepted for API parity; RCCL picks ring/tree channels
itself over the 7 xGMI links.
"""
from __future__ import annotations

import operator
import os
from typing import Any, Callable, Dict, List, Optional, Tuple

import torch

from ..ops.flat import HEADER, SLOT, fill_
from ..utils.walk import walk_table
from .comm import Communicator, init_communicator


class FlatBuffer:
    """A flat 1-D buffer with the participation header (zero-copy allReduce)."""

    def __init__(self, buf: torch.Tensor):
        if buf.dim() != 1 or buf.numel() < HEADER:
            raise ValueError("FlatBuffer needs a 1-D tensor with a header")
        self.buf = buf

    def tensors(self):
        return [self.buf]

    @property
    def slot(self) -> torch.Tensor:
        return self.buf[SLOT:SLOT + 1]


_SUM_ALIASES = {None, "sum", "add", "+"}


def _classify_op(op) -> Optional[str]:
    """Map a user reduction to a native op name, or None for a generic op.

    The reference passes Lua closures ``function(a, b) return a:add(b) end``;
    Python callers pass e.g. ``lambda a, b: a.add_(b)``.  Known callables are
    recognised directly; unknown ones are probed on a tiny CPU tensor.
    """
    if op in _SUM_ALIASES or op is torch.add or op is operator.add or op is operator.iadd:
        return "sum"
    if op in ("max", "min", "prod"):
        return op
    if op is torch.max or op is torch.maximum:
        return "max"
    if op is torch.min or op is torch.minimum:
        return "min"
    if callable(op):
        a = torch.tensor([1.0, -2.0, 3.5], dtype=torch.float64)
        b = torch.tensor([2.0, 4.0, -1.0], dtype=torch.float64)
        try:
            r = op(a.clone(), b.clone())
        except Exception:
            return None
        if not isinstance(r, torch.Tensor):
            return None
        for name, ref in (("sum", a + b), ("max", torch.maximum(a, b)), ("min", torch.minimum(a, b)),
                          ("prod", a * b)):
            if r.shape == ref.shape and torch.equal(r, ref):
                return name
        return None
    raise TypeError(f"unsupported reduction op {op!r}")


class Tree:
    """Collective topology object (``ipc.Tree`` contract) over RCCL/gloo."""

    def __init__(self, nodeIndex: Optional[int] = None, numNodes: Optional[int] = None, base: int = 2,
                 server: Any = None, client: Any = None, host: Optional[str] = None, port: Optional[int] = None,
                 device=None, backend: str = "auto", comm: Optional[Communicator] = None):
        if comm is None:
            rank = None if nodeIndex is None else int(nodeIndex) - 1
            comm = init_communicator(rank=rank, world_size=numNodes, host=host, port=port, device=device,
                                     backend=backend)
        self.comm = comm
        self.nodeIndex = comm.rank + 1  # 1-based like the reference (root = node 1)
        self.numNodes = comm.world_size
        self.base = base
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._staging: Dict[Tuple, torch.Tensor] = {}
        self._last_layout: Optional[List[torch.Tensor]] = None
        self.walkTable = walk_table

    # python spellings
    @property
    def rank(self) -> int:
        return self.comm.rank

    @property
    def world_size(self) -> int:
        return self.comm.world_size

    # ------------------------------------------------------------------
    def _stage(self, key, numel, dtype, device) -> torch.Tensor:
        buf = self._staging.get(key)
        if buf is None or buf.numel() < numel:
            buf = torch.zeros(numel, dtype=dtype, device=device)
            self._staging[key] = buf
        return buf[:numel]

    def _groups(self, leaves: List[torch.Tensor]):
        groups: Dict[Tuple, List[int]] = {}
        for i, t in enumerate(leaves):
            groups.setdefault((t.device.type, t.device.index, t.dtype), []).append(i)
        return groups

    def _round(self, leaves: List[torch.Tensor], participating: bool, opname: str,
               outs: Optional[List[torch.Tensor]] = None):
        """One collective round over ``leaves``; results land in ``outs``
        (default: in place).  Returns n (device tensor for flat GPU buffers,
        python int otherwise)."""
        outs = leaves if outs is None else outs
        comm = self.comm
        # ---- zero-copy flat buffer ------------------------------------------------
        if len(leaves) == 1 and getattr(leaves[0], "_dl_flat", False):
            buf = leaves[0]
            buf[SLOT:SLOT + 1].fill_(1 if participating else 0)  # a fill kernel: capturable in a hipGraph
            if opname == "sum":
                comm.all_reduce(buf, "sum")
            else:
                cnt = buf[SLOT:SLOT + 1].clone()
                comm.all_reduce(buf, opname)
                comm.all_reduce(cnt, "sum")
                buf[SLOT] = cnt[0]
            if outs[0] is not buf:
                outs[0].copy_(buf)
            return buf[SLOT]
        # ---- generic table: pack per (device, dtype) ------------------------------------
        groups = self._groups(leaves)
        staged = []
        for gi, (key, idxs) in enumerate(sorted(groups.items(), key=lambda kv: kv[1][0])):
            total = HEADER + sum(leaves[i].numel() for i in idxs)
            t0 = leaves[idxs[0]]
            buf = self._stage(key, total, t0.dtype, t0.device)
            buf[:HEADER].zero_()
            if gi == 0:
                buf[SLOT:SLOT + 1].fill_(1 if participating else 0)
            off = HEADER
            views = []
            for i in idxs:
                n = leaves[i].numel()
                views.append(buf[off:off + n])
                off += n
            if t0.is_cuda:
                torch._foreach_copy_(views, [leaves[i].reshape(-1) for i in idxs])
            else:
                for v, i in zip(views, idxs):
                    v.copy_(leaves[i].reshape(-1))
            staged.append((buf, idxs, views))
        count_buf = staged[0][0][SLOT:SLOT + 1]
        cnt = None
        if opname != "sum":
            cnt = count_buf.clone()
        with comm.group():
            for buf, _, _ in staged:
                comm.all_reduce(buf, opname)
        if cnt is not None:
            comm.all_reduce(cnt, "sum")
            count_buf.copy_(cnt)
        for buf, idxs, views in staged:
            if buf.is_cuda:
                torch._foreach_copy_([outs[i].view(-1) for i in idxs], views)
            else:
                for v, i in zip(views, idxs):
                    outs[i].view(-1).copy_(v)
        n = staged[0][0][SLOT]
        return n if n.is_cuda else int(n.item())

    def _generic_round(self, leaves, participating, op, outs=None):
        """Arbitrary user op: all-gather every contribution and fold with ``op``
        in node order (deterministic, identical on all nodes)."""
        outs = leaves if outs is None else outs
        W = self.comm.world_size
        flags = torch.tensor([1 if participating else 0], dtype=torch.int64)
        self.comm.all_reduce_host(flags, "sum")
        for t, o in zip(leaves, outs):
            flat = t.reshape(-1).contiguous()
            gathered = torch.empty(W * flat.numel(), dtype=flat.dtype, device=flat.device)
            self.comm.all_gather(gathered, flat)
            parts = gathered.view(W, -1)
            acc = parts[0].clone()
            for r in range(1, W):
                acc = op(acc, parts[r].clone())
            o.view(-1).copy_(acc)
        return int(flags.item())

    # ------------------------------------------------------------------ API
    def allReduce(self, value: Any, op: Any = None, zero: Optional[Callable] = None):  # noqa: N802
        opname = _classify_op(op)
        if zero is None:
            leaves = self._leaves(value)
            self._last_layout = leaves
            if opname is None:
                n = self._generic_round(leaves, True, op)
            else:
                n = self._round(leaves, True, opname)
            return value, n
        # ---- drain -----------------------------------------------------------------
        leaves = self._leaves(value) if value is not None else self._drain_layout()
        while True:
            contribs = []
            for i, t in enumerate(leaves, 1):
                r = zero(t, i)
                contribs.append(r if isinstance(r, torch.Tensor) else t)
            if opname is None:
                n = self._generic_round(contribs, False, op, outs=leaves)
            else:
                n = self._round(contribs, False, opname, outs=leaves)
            n = int(n.item()) if isinstance(n, torch.Tensor) else int(n)
            if n == 0:
                return value, n

    def _leaves(self, value) -> List[torch.Tensor]:
        if isinstance(value, FlatBuffer):
            value.buf._dl_flat = True
            return [value.buf]
        leaves = walk_table(value)
        if not leaves:
            raise ValueError("allReduce: value has no tensors")
        return leaves

    def _drain_layout(self) -> List[torch.Tensor]:
        if self._last_layout is None:
            raise RuntimeError("allReduce(nil, op, zero): no previous layout to drain with")
        out = []
        for t in self._last_layout:
            z = torch.zeros_like(t)
            if getattr(t, "_dl_flat", False):
                z._dl_flat = True
            out.append(z)
        return out

    def scatter(self, value: Any, root: int = 0):
        """Broadcast ``value`` in place from node ``root+1`` (reference: root = node 1)."""
        for t in self._leaves(value):
            self.comm.broadcast(t, root)
        return value

    def broadcast(self, value: Any, root: int):
        return self.scatter(value, root)


def LocalhostTree(nodeIndex: int, numNodes: int, port: Optional[int] = None, device=None,  # noqa: N802
                  backend: str = "auto", base: int = 2) -> Tree:
    """All nodes on one host (examples/mnist.lua:16); rendezvous on 127.0.0.1."""
    port = port or int(os.environ.get("DISTLEARN_PORT", os.environ.get("MASTER_PORT", "8080")))
    return Tree(nodeIndex, numNodes, base=base, host="127.0.0.1", port=port, device=device, backend=backend)
