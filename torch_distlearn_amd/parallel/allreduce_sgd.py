"""AllReduceSGD: synchronous data parallelism with uneven-step handling.

Reference: lua/AllReduceSGD.lua:1-63 (API ``sumGradients``,
``sumAndNormalizeGradients``, ``synchronizeParameters``, exported at :56-60).

Semantics kept exactly:

* ``sumGradients(grads)`` -- all-reduce (sum) the gradients in place and count
  one step for this node (:10-15).
* ``sumAndNormalizeGradients(grads)`` -- all-reduce, then divide by the
  number ``n`` of nodes that *contributed this round* when ``n > 1`` (:18-30);
  "not all nodes contribute to every step due to uneven partitioning of data".
* ``synchronizeParameters(params)`` -- after uneven epochs, keep joining the
  still-active nodes' all-reduces with zero contributions until every node has
  finished, all-reduce the per-node step counts, and give every node the
  parameters of the node with the most steps (:33-54).

MI355X design:

* When ``grads``/``params`` are a :class:`FlatParams` (or its buffers), the
  all-reduce is zero-copy on the persistent flat buffer and ``n`` is carried in
  the buffer's participation slot; normalisation is a device kernel that reads
  ``n`` on the GPU (no host sync), and :meth:`step` fuses 1/n into the SGD
  update (one HIP kernel over the whole model, csrc/kernels/flat_ops.hip).
* With a :class:`~torch_distlearn_amd.parallel.buckets.GradBucketer` attached,
  gradients are all-reduced in buckets on a side stream *during backward*;
  a draining node replays the same bucket sequence with zeros.
* The winner's parameters are sent with one broadcast from the winner
  (bitwise identical to the reference's all-reduce of zeros + winner, and
  half the traffic).
* Reference bug fixed (SURVEY §3.3 "edge case"): a node with 0 steps used to
  ``scatter`` while others drained -> deadlock.  Here every node drains first,
  so the collective sequence is identical on all nodes.
"""
from __future__ import annotations

from typing import Any, Optional

import torch

from ..ops.flat import HEADER, FlatParams, flat_sgd_, scale_by_count_, sgd_update_
from ..utils.walk import walk_table
from .tree import FlatBuffer, Tree


def _flat_of(x) -> Optional[FlatParams]:
    return x if isinstance(x, FlatParams) else None


class AllReduceSGD:
    """``AllReduceSGD(tree)`` (lua/AllReduceSGD.lua:3)."""

    def __init__(self, tree: Tree, bucketer=None):
        self.tree = tree
        self.stepsPerNode = torch.zeros(tree.numNodes, dtype=torch.int64)  # :7 (host, like LongTensor)
        self.bucketer = bucketer
        self._drain_template = None

    # ------------------------------------------------------------ internals
    def _grad_value(self, grads):
        f = _flat_of(grads)
        if f is not None:
            return FlatBuffer(f.grad)
        return grads

    def _count_step(self):
        self.stepsPerNode[self.tree.nodeIndex - 1] += 1

    # ------------------------------------------------------------------ API
    def _no_bucket_updates(self, what: str) -> None:
        if self.bucketer is not None and self.bucketer.early is not None:
            raise RuntimeError(f"{what}: the bucketer updates parameters per bucket (enable_bucket_updates); "
                               "use step()")

    def sumGradients(self, grads: Any) -> None:  # noqa: N802  (:10-15)
        self._no_bucket_updates("sumGradients")
        if self.bucketer is not None and _flat_of(grads) is self.bucketer.flat:
            self.bucketer.finish()
        else:
            self.tree.allReduce(self._grad_value(grads))
            self._remember(grads)
        self._count_step()

    def sumAndNormalizeGradients(self, grads: Any) -> None:  # noqa: N802  (:18-30)
        self._no_bucket_updates("sumAndNormalizeGradients")
        f = _flat_of(grads)
        if self.bucketer is not None and f is self.bucketer.flat:
            self.bucketer.finish()
            scale_by_count_(f.grad[HEADER:], f.slot)  # the header (slot) itself is never scaled
        elif f is not None:
            self.tree.allReduce(FlatBuffer(f.grad))
            scale_by_count_(f.grad[HEADER:], f.slot)
        else:
            _, n = self.tree.allReduce(grads)
            leaves = walk_table(grads)
            if isinstance(n, torch.Tensor):  # GPU generic path: keep n on the device
                s = torch.where(n > 1, 1.0 / n.float(), torch.ones_like(n, dtype=torch.float32))
                for t in leaves:
                    t.mul_(s.to(t.dtype))
            elif n > 1:
                for t in leaves:
                    t.mul_(1.0 / n)
        self._remember(grads)
        self._count_step()

    def step(self, flat: FlatParams, lr: float, momentum: float = 0.0, weight_decay: float = 0.0,
             momentum_buf: Optional[torch.Tensor] = None, already_reduced: bool = False, slabs=None,
             skip=None) -> None:
        """Fused ``sumAndNormalizeGradients`` + SGD update over a FlatParams:
        all-reduce (unless the bucketer already did), then ONE kernel
        ``p -= lr*(g/n + wd*p)`` (+momentum, + bf16 shadow refresh).  This is
        examples/cifar10.lua:184-191 in one launch.  ``slabs`` (one node
        only: nothing is all-reduced): leaves whose gradient the update sums
        from split-K slabs itself (ops/flat.py flat_sgd_); ``skip``: a flat
        element range [lo, hi) already updated inside the step (a conv
        launch's side job)."""
        if (slabs or skip) and self.tree.numNodes > 1:
            raise ValueError("AllReduceSGD.step: slab gradients are never all-reduced (one node only)")
        g = None
        bk = self.bucketer if (self.bucketer is not None and flat is self.bucketer.flat) else None
        if not already_reduced:
            if bk is not None:
                bk.finish(widen=False)  # bf16 wire: the update reads the reduced bf16 copy directly
            else:
                self.tree.allReduce(FlatBuffer(flat.grad))
            self._count_step()
            self._remember(flat)
        if bk is not None and not already_reduced and bk.early_applied:
            return  # every bucket was updated on the comm stream right after its all-reduce
        if bk is not None and bk.wire16 and not already_reduced:
            g = flat.grad16
        flat_sgd_(flat, lr, slot=flat.slot, mom=momentum_buf, momentum=momentum, weight_decay=weight_decay, grad=g,
                  slabs=slabs, skip=skip)

    def enable_bucket_updates(self, flat: FlatParams, lr_fn, momentum: float = 0.0, weight_decay: float = 0.0,
                              momentum_buf: Optional[torch.Tensor] = None) -> bool:
        """Fold the fused SGD of :meth:`step` into the bucketer: each bucket's
        parameters are updated on the comm stream right after its all-reduce
        (buckets.py set_early_update).  ``lr_fn()`` returns the current rate.
        Only for callers whose backward never reads a parameter after its
        bucket is complete (the HIP executors).  Returns whether it is on."""
        bk = self.bucketer
        if bk is None or flat is not bk.flat:
            return False

        def update(s: int, e: int, g: torch.Tensor) -> None:
            sgd_update_(flat.data[s:e], g[s:e], lr_fn(), slot=flat.slot,
                        mom=None if momentum_buf is None else momentum_buf[s:e], momentum=momentum,
                        weight_decay=weight_decay, shadow=None if flat.shadow is None else flat.shadow[s:e])

        bk.set_early_update(update)
        return True

    def _remember(self, grads):
        if self._drain_template is None:
            f = _flat_of(grads)
            if f is not None:
                self._drain_template = ("flat", f)
            else:
                self._drain_template = ("table", [torch.zeros_like(t) for t in walk_table(grads)])

    def _drain(self, params):
        """Contribute zeros until every node is draining (reference :37)."""
        if self.bucketer is not None:
            self.bucketer.drain()
            return
        tmpl = self._drain_template
        if tmpl is None:  # never stepped: grads have the shapes of params
            f = _flat_of(params)
            tmpl = ("flat", f) if f is not None else ("table", [torch.zeros_like(t) for t in walk_table(params)])
            self._drain_template = tmpl
        if tmpl[0] == "flat":
            f = tmpl[1]
            value = FlatBuffer(torch.zeros_like(f.grad))
        else:
            value = tmpl[1]
        self.tree.allReduce(value, "sum", lambda a, i=None: a.zero_())

    def synchronizeParameters(self, params: Any) -> Any:  # noqa: N802  (:33-54)
        # 1. drain (all nodes, deadlock-free even with zero-step nodes)
        self._drain(params)
        from ..utils.debug import check_collective_sequence

        check_collective_sequence(self.tree, "synchronizeParameters")  # DISTLEARN_DEBUG_SYNC=1
        # 2. everybody learns everybody's step count (:39); control plane
        steps = self.stepsPerNode.clone()
        self.tree.comm.all_reduce_host(steps, "sum")
        value = params.data if isinstance(params, FlatParams) else params
        if isinstance(params, FlatParams):
            value = FlatBuffer(params.data)
        if int(steps.sum()) == 0:
            # first call / no training: scatter root's params (:52)
            self.tree.scatter(value, 0)
        else:
            # 3. the node with the most steps saw every round's update (:41-47);
            #    ties -> lowest index (all tied nodes hold identical params)
            winner = int(torch.argmax(steps).item())
            self.tree.broadcast(value, winner)
        if isinstance(params, FlatParams):
            params.refresh_shadow()
        self.stepsPerNode.zero_()  # (:49)
        from ..utils.debug import assert_replicas_in_sync, debug_sync_enabled

        if debug_sync_enabled():
            assert_replicas_in_sync(self.tree, params.data if isinstance(params, FlatParams)
                                    else torch.cat([t.reshape(-1) for t in walk_table(params)]))
        return params

    # python spellings
    sum_gradients = sumGradients
    sum_and_normalize_gradients = sumAndNormalizeGradients
    synchronize_parameters = synchronizeParameters
