"""AllReduceEA: synchronous Elastic-Averaging SGD (arXiv:1412.6651).

Reference: lua/AllReduceEA.lua:1-109, design note lua/AllReduceEA.md:12-30.
Every node keeps a replica of the center variable ``c``.  Every ``tau`` steps:

    delta = alpha * (p - c);  p -= delta;  allReduce(delta);  c += sum(delta)

so one averaging round is ONE all-reduce of a params-sized buffer (the
reference's whole point, AllReduceEA.md:12-24).

MI355X design: parameters, center and delta live in persistent flat buffers
(:class:`FlatParams` layout, user tensors are re-pointed into the flat
parameter buffer), the elastic move is one fused HIP kernel writing delta
straight into the communication buffer (csrc/kernels/flat_ops.hip
``elastic_kernel``), the all-reduce is one zero-copy RCCL call carrying the
participation count in its header, and the drain step of
``handleUnevenSteps`` (c += sum(delta); delta = alpha(p-c); p -= delta) is the
same kernel with the ``pending`` input (K10, one launch per drain round).

Reference issues handled:
* ``flatParam`` cached stale tensor objects when the example replaced params
  out of place: here every call re-checks that the user's
  leaves still alias the flat buffer and re-points/copies them if not.
* a node with 0 steps skipped the drain (``if step > 0``) and scattered while
  others were still averaging -> deadlock; every node drains here (a round in
  which all nodes drain ends immediately with n == 0).
"""
from __future__ import annotations

from typing import Any, Optional

import torch

from ..ops.flat import HEADER, FlatParams, add_, elastic_step_
from ..utils.walk import walk_table
from .tree import FlatBuffer, Tree


class _FlatState:
    """Flat storage bound to a user parameter table."""

    def __init__(self, params: Any, shadow: bool = False):
        if isinstance(params, FlatParams):
            self.flat = params
            self.owned = False
        else:
            self.flat = FlatParams(params, grads=False, shadow_bf16=shadow)
            self.owned = True

    def sync_in(self, params: Any) -> None:
        """Make sure every user leaf aliases the flat buffer (copy if replaced)."""
        if isinstance(params, FlatParams):
            return
        leaves = walk_table(params)
        views = self.flat.param_views()
        if len(leaves) != len(views):
            raise ValueError("AllReduceEA: parameter table changed structure")
        storage = self.flat.data.untyped_storage()
        for t, v, off, shape in zip(leaves, views, self.flat.offsets, self.flat.shapes):
            if t.data_ptr() != v.data_ptr():
                with torch.no_grad():
                    v.copy_(t.reshape(v.shape))
                    t.set_(storage, off, shape, v.stride())


class AllReduceEA:
    """``AllReduceEA(tree, tau, alpha)`` (lua/AllReduceEA.lua:2)."""

    def __init__(self, tree: Tree, tau: int, alpha: float):
        self.tree = tree
        self.tau = int(tau)
        self.alpha = float(alpha)
        self.step = 0
        self.state: Optional[_FlatState] = None
        self.center: Optional[torch.Tensor] = None
        self.delta: Optional[torch.Tensor] = None

    def _one_time_init(self, params: Any) -> None:  # (:11-22)
        if self.state is None:
            self.state = _FlatState(params)
            f = self.state.flat
            self.center = f.data.clone()
            self.delta = f.data.clone()
        else:
            self.state.sync_in(params)

    @property
    def flat(self) -> FlatParams:
        return self.state.flat

    def averageParameters(self, params: Any) -> bool:  # noqa: N802  (:25-47)
        """Returns True when an averaging round ran this call."""
        self._one_time_init(params)
        self.step += 1
        if self.step % self.tau != 0:
            return False
        self.elastic_round()
        return True

    def elastic_round(self) -> None:
        """The averaging round's device work, no host synchronisation (also
        captured into the engine's tau-step hipGraph)."""
        p, c, d, s = self._body()
        # delta = alpha (p - c); p -= delta   (K8, writes the comm buffer)
        elastic_step_(p, c, d, self.alpha, shadow=s)
        self.tree.allReduce(FlatBuffer(self.delta))  # (:41)
        add_(c, d)                                   # c += sum(delta)  (:43-45)

    def _body(self):
        """(params, center, delta, shadow) without the 64-element header: the
        delta buffer's header carries the all-reduced participation count,
        which must never flow into the center or the parameters."""
        f = self.flat
        return (f.data[HEADER:], self.center[HEADER:], self.delta[HEADER:],
                None if f.shadow is None else f.shadow[HEADER:])

    def _handle_uneven_steps(self) -> None:  # (:50-72)
        p, c, d, s = self._body()
        self.delta.zero_()
        rounds = [0]
        idle = self.step == 0

        def drain_step(_t, _i):
            rounds[0] += 1
            if rounds[0] == 1 and idle:
                # reference guard ``if step > 0`` (:52): a node with no pending
                # steps contributes zeros and does not move in the first round;
                # if every node is idle that round ends the drain (n == 0) and
                # params are untouched.  It still joins the rounds, so a mix of
                # idle and active nodes cannot deadlock (the reference did).
                return self.delta
            # c += previous round's sum(delta); delta = alpha (p - c); p -= delta   (K10)
            elastic_step_(p, c, d, self.alpha, pending=d, shadow=s)
            return self.delta

        self.tree.allReduce(FlatBuffer(self.delta), "sum", drain_step)
        self.step = 0
        from ..utils.debug import check_collective_sequence

        check_collective_sequence(self.tree, "the AllReduceEA epoch synchronisation")  # DISTLEARN_DEBUG_SYNC=1

    def synchronizeCenter(self, params: Any) -> Any:  # noqa: N802  (:77-84)
        self._one_time_init(params)
        self._handle_uneven_steps()
        self.tree.scatter(FlatBuffer(self.center))  # centers bit-identical despite FP drift (:74-76)
        return params

    def synchronizeParameters(self, params: Any) -> Any:  # noqa: N802  (:87-100)
        self._one_time_init(params)
        self._handle_uneven_steps()
        f = self.flat
        self.tree.scatter(FlatBuffer(f.data))
        self.center.copy_(f.data)
        f.refresh_shadow()
        return params

    average_parameters = averageParameters
    synchronize_center = synchronizeCenter
    synchronize_parameters = synchronizeParameters
