"""Flat persistent parameter/gradient storage and the fused flat-bucket ops.

``FlatParams`` is the MI355X analogue of torch-autograd's ``stableGradients``
(examples/mnist.lua:91-94: "Keep the gradient tensors stable so we can use
CUDA IPC"): every parameter and gradient of a table/module becomes a *view*
into one contiguous, 256-byte aligned buffer, so

  * a collective over all gradients is one (or a few, bucketed) RCCL calls on
    the flat buffer -- no per-tensor walkTable serialisation;
  * the reference's per-tensor update loops (K3/K5/K8/K9/K10) become single
    fused HIP kernels over the flat buffer (csrc/kernels/flat_ops.hip);
  * tensor objects never move, which also fixes the reference hazard where
    AllReduceEA caches tensor objects that the example then replaces
    (lua/AllReduceEA.lua:19 vs examples/mnist-ea.lua:103-107).

The grad buffer reserves a 64-element header whose element 0 is the
*participation slot*: each node writes 1 (normal step) or 0 (draining), and
the all-reduced value is the reference's ``n`` (lua/AllReduceSGD.lua:20-27),
delivered by the same collective at no extra latency.
"""
from __future__ import annotations

from typing import Any, List, Sequence, Tuple

import torch

from .._native import native, stream_handle
from ..utils.walk import walk_table

ALIGN = 64        # elements; 256 B for fp32 -> every view is 16-B aligned for float4 kernels
HEADER = 64       # reserved elements at the start of the grad/delta buffers
SLOT = 0          # participation slot index inside the header


def _round_up(x: int, a: int) -> int:
    return (x + a - 1) // a * a


class FlatParams:
    """Persistent flat storage for a (nested) parameter table or nn.Module.

    Args:
        params: tensor table or ``nn.Module``; its leaves are re-pointed (``set_``)
            into the flat buffer, so existing references stay valid.
        grads: also allocate a flat gradient buffer (with participation header);
            for ``nn.Parameter`` leaves ``p.grad`` becomes the matching view.
        shadow_bf16: keep a bf16 copy of the parameters (refreshed by the fused
            update kernels) for the bf16 compute path.
    """

    def __init__(self, params: Any, grads: bool = True, shadow_bf16: bool = False, device=None):
        self.table = params
        leaves = walk_table(params)
        if not leaves:
            raise ValueError("FlatParams: empty parameter table")
        dtype = leaves[0].dtype
        if any(t.dtype != dtype for t in leaves):
            raise ValueError("FlatParams: all leaves must share one dtype")
        self.dtype = dtype
        self.device = torch.device(device) if device is not None else leaves[0].device
        self.shapes = [tuple(t.shape) for t in leaves]
        self.numels = [t.numel() for t in leaves]
        offs, o = [], HEADER
        for n in self.numels:
            offs.append(o)
            o = _round_up(o + n, ALIGN)
        self.offsets = offs
        self.total = o  # includes header + padding, multiple of ALIGN
        self.numel = sum(self.numels)
        self.data = torch.zeros(self.total, dtype=dtype, device=self.device)
        with torch.no_grad():
            for t, off, n in zip(leaves, offs, self.numels):
                self.data[off:off + n].copy_(t.reshape(-1))
            for t, off, shape in zip(leaves, offs, self.shapes):
                t.set_(self.data.untyped_storage(), off, shape, _contig_stride(shape))
        self.leaves = leaves
        self.grad = None
        if grads:
            self.grad = torch.zeros(self.total, dtype=dtype, device=self.device)
            self.grad_views = self._views(self.grad)
            for t, g in zip(leaves, self.grad_views):
                if isinstance(t, torch.nn.Parameter) or t.requires_grad:
                    t.grad = g
        self.shadow = None
        if shadow_bf16:
            self.shadow = torch.zeros(self.total, dtype=torch.bfloat16, device=self.device)
            self.refresh_shadow()
        self.grad16 = None  # bf16 wire copy of the gradient (enable_grad16)

    def enable_grad16(self) -> torch.Tensor:
        """Allocate the bf16 gradient wire buffer (same layout as ``grad``):
        with ``grad_comm_dtype="bf16"`` the bucketed all-reduce sends this
        copy -- half the xGMI bytes -- and the fused SGD reads it directly;
        the participation count stays fp32 (``grad``'s header, all-reduced
        beside it in the same group)."""
        if self.grad is None:
            raise ValueError("FlatParams.enable_grad16: no gradient buffer")
        if self.grad16 is None:
            self.grad16 = torch.zeros(self.total, dtype=torch.bfloat16, device=self.device)
        return self.grad16

    # ----------------------------------------------------------------- views
    def _views(self, buf: torch.Tensor) -> List[torch.Tensor]:
        return [buf[o:o + n].view(s) for o, n, s in zip(self.offsets, self.numels, self.shapes)]

    def param_views(self) -> List[torch.Tensor]:
        return self._views(self.data)

    def like(self, fill: float = 0.0, dtype=None) -> torch.Tensor:
        """A new flat buffer with the same layout (e.g. EA center/delta)."""
        return torch.full((self.total,), fill, dtype=dtype or self.dtype, device=self.device)

    def views_of(self, buf: torch.Tensor) -> List[torch.Tensor]:
        return self._views(buf)

    def shadow_views(self) -> List[torch.Tensor]:
        assert self.shadow is not None
        return self._views(self.shadow)

    def tensors(self):  # lets walk_table() visit a FlatParams
        return self.leaves

    # -------------------------------------------------------------- buckets
    def buckets(self, bucket_bytes: int) -> List[Tuple[int, int]]:
        """Contiguous [start, end) ranges of the flat buffer in *reverse*
        registration order (backward produces the last layers' grads first),
        each at least ``bucket_bytes`` unless it is the last; boundaries fall
        on tensor boundaries; the first range issued last includes the header
        (participation slot) so ``n`` is complete when the last bucket lands."""
        limit = max(1, bucket_bytes // self.data.element_size())
        out: List[Tuple[int, int]] = []
        end = self.total
        for i in reversed(range(len(self.offsets))):
            start = self.offsets[i] if i > 0 else 0
            if end - start >= limit or i == 0:
                out.append((start, end))
                end = start
        return out

    # ---------------------------------------------------------------- misc
    def refresh_shadow(self) -> None:
        if self.shadow is None:
            return
        if self.data.is_cuda:
            native().cast_f32_bf16(self.data.data_ptr(), self.shadow.data_ptr(), self.total, stream_handle())
        else:
            self.shadow.copy_(self.data)

    def zero_grad(self, participating: bool = True) -> None:
        fill_(self.grad, 0.0, slot_value=1.0 if participating else 0.0)

    @property
    def slot(self) -> torch.Tensor:
        return self.grad[SLOT:SLOT + 1]


def _contig_stride(shape: Sequence[int]) -> Tuple[int, ...]:
    st, acc = [], 1
    for s in reversed(shape):
        st.append(acc)
        acc *= max(1, s)
    return tuple(reversed(st))


# ---------------------------------------------------------------------------
# fused flat ops: HIP on GPU (native, loud failure if missing), torch on CPU
# ---------------------------------------------------------------------------
def _ptr(t):
    return 0 if t is None else t.data_ptr()


def _scale_from_slot(slot):
    if slot is None:
        return 1.0
    n = float(slot.reshape(-1)[0])
    return 1.0 / n if n > 1 else 1.0


def sgd_update_(p: torch.Tensor, g: torch.Tensor, lr: float, slot: torch.Tensor | None = None,
                mom: torch.Tensor | None = None, momentum: float = 0.0, weight_decay: float = 0.0,
                shadow: torch.Tensor | None = None, slabs=None, tail=None, skip=None) -> None:
    """p -= lr * (g/n + wd*p) [with momentum buffer]; n from ``slot`` (device).
    ``g`` is fp32, or bf16 (the all-reduced wire copy of grad_comm_dtype="bf16").
    ``slabs``: [(offset into p, numel, slab tensor [splits * numel], splits)]:
    in those ranges the gradient is the sum of the split-K slabs instead of
    ``g`` (one GPU: the conv executor's deferred slab reduce; bitwise the
    stand-alone reduce's sum).  ``tail``: one channel-padded range
    (offset, numel, slab tensor, splits, Cout, taps, Cp, C) reduced by extra
    blocks of the same launch.  ``skip``: elements [lo, hi) of p left alone
    (updated inside the step by a conv launch's side job)."""
    # an armed next-step preparation (executor arm_next_prep) rides the slab-capable launch
    armed = p.is_cuda and native().sgd_next_prep_armed()
    if slabs or tail is not None or skip is not None or armed:
        if not p.is_cuda or g.dtype != torch.float32:
            raise ValueError("sgd_update_: slab gradients / the next-step preparation need an fp32 gradient "
                             "on the GPU")
        slabs = slabs or []
        tl, tptr = [], 0
        if tail is not None:
            o, n, t, k, cout, taps, cp, c = tail
            tl, tptr = [int(o), int(n), int(k), int(cout), int(taps), int(cp), int(c)], t.data_ptr()
        native().sgd_update_slabs(p.data_ptr(), g.data_ptr(), _ptr(mom), _ptr(shadow), _ptr(slot), float(lr),
                                  float(momentum), float(weight_decay), p.numel(), [int(o) for o, _, _, _ in slabs],
                                  [int(n) for _, n, _, _ in slabs], [t.data_ptr() for _, _, t, _ in slabs],
                                  [int(k) for _, _, _, k in slabs], tl, tptr,
                                  int(skip[0]) if skip else 0, int(skip[1]) if skip else 0, stream_handle())
        return
    if p.is_cuda:
        fn = native().sgd_update_g16 if g.dtype == torch.bfloat16 else native().sgd_update
        fn(p.data_ptr(), g.data_ptr(), _ptr(mom), _ptr(shadow), _ptr(slot), float(lr), float(momentum),
           float(weight_decay), p.numel(), stream_handle())
        return
    with torch.no_grad():
        d = g.float() * _scale_from_slot(slot)
        if weight_decay:
            d = d + weight_decay * p
        if mom is not None:
            mom.mul_(momentum).add_(d)
            d = mom
        p.sub_(lr * d)
        if shadow is not None:
            shadow.copy_(p)


def _overlaps(x: torch.Tensor, y: torch.Tensor) -> bool:
    if x.untyped_storage().data_ptr() != y.untyped_storage().data_ptr():
        return False
    xs, ys = x.data_ptr(), y.data_ptr()
    return xs < ys + y.numel() * y.element_size() and ys < xs + x.numel() * x.element_size()


def flat_sgd_(flat: "FlatParams", lr: float, slot: torch.Tensor | None = None, mom: torch.Tensor | None = None,
              momentum: float = 0.0, weight_decay: float = 0.0, grad: torch.Tensor | None = None,
              slabs=None, skip=None) -> None:
    """The fused update over a FlatParams' parameter body: the 64-element
    header (whose gradient element is the participation count) is left out,
    so ``n`` never flows into the parameter buffer.  ``grad``: the gradient
    buffer to read (default ``flat.grad``; ``flat.grad16`` for bf16 comm).
    ``slabs``: [(leaf index, slab tensor, splits, Cout, taps, Cp, C)] whose
    gradient is still in split-K slabs [splits][Cout][taps][Cp] (see
    :func:`sgd_update_`): unpadded ones (Cp == C) with < 32 splits are read
    in place, at most one other is reduced by extra blocks of the launch.
    ``skip``: a flat element range [lo, hi) (offsets into ``flat.data``)
    already updated inside the step."""
    H = HEADER
    g = flat.grad if grad is None else grad
    rng, tail = None, None
    if slabs:
        rng = []
        for i, t, k, cout, taps, cp, c in slabs:
            off, n = flat.offsets[i] - H, flat.numels[i]
            if n != cout * taps * c:
                raise ValueError("flat_sgd_: slab layout does not match the leaf")
            if cp == c and k < 32:
                rng.append((off, n, t, k))
            elif tail is None:
                tail = (off, n, t, k, cout, taps, cp, c)
            else:
                raise ValueError("flat_sgd_: at most one channel-padded slab range")
        rng.sort(key=lambda r: r[0])
    sgd_update_(flat.data[H:], g[H:], lr, slot=slot, mom=None if mom is None else mom[H:],
                momentum=momentum, weight_decay=weight_decay,
                shadow=None if flat.shadow is None else flat.shadow[H:], slabs=rng, tail=tail,
                skip=None if skip is None else (max(0, skip[0] - H), skip[1] - H))


def scale_by_count_(x: torch.Tensor, slot: torch.Tensor) -> None:
    """x *= 1/n with n read from ``slot`` on the device.  ``slot`` must not lie
    inside ``x`` (every workgroup reads n; one that ran after the slot's own
    element was scaled would read 1): scale ``grad[HEADER:]``."""
    if _overlaps(x, slot):
        raise ValueError("scale_by_count_: the slot lies inside the scaled buffer (pass grad[HEADER:])")
    if x.is_cuda:
        native().scale_by_count(x.data_ptr(), slot.data_ptr(), x.numel(), stream_handle())
        return
    s = _scale_from_slot(slot)
    if s != 1.0:
        x.mul_(s)


def elastic_step_(p: torch.Tensor, c: torch.Tensor, out: torch.Tensor, alpha: float,
                  pending: torch.Tensor | None = None, shadow: torch.Tensor | None = None) -> None:
    """[c += pending]; out = alpha*(p - c); p -= out   (K8, fused K10)."""
    if p.is_cuda:
        native().elastic_step(p.data_ptr(), c.data_ptr(), _ptr(pending), out.data_ptr(), _ptr(shadow),
                              float(alpha), p.numel(), stream_handle())
        return
    with torch.no_grad():
        if pending is not None:
            c.add_(pending)
        torch.sub(p, c, out=out)
        out.mul_(alpha)
        p.sub_(out)
        if shadow is not None:
            shadow.copy_(p)


def elastic_step_wire16_(p: torch.Tensor, c: torch.Tensor, out: torch.Tensor, out16: torch.Tensor,
                         alpha: float, shadow: torch.Tensor | None = None) -> None:
    """AsyncEA bf16 delta wire: out16 = bf16(alpha*(p - c)); out = float(out16);
    p -= out (the ROUNDED delta: p + c conserved); [shadow = bf16(p)]."""
    if p.is_cuda and p.numel() % 4 == 0:
        native().elastic_step_wire16(p.data_ptr(), c.data_ptr(), out.data_ptr(), out16.data_ptr(), _ptr(shadow),
                                     float(alpha), p.numel(), stream_handle())
        return
    with torch.no_grad():
        torch.sub(p, c, out=out)
        out.mul_(alpha)
        out16.copy_(out)
        out.copy_(out16)
        p.sub_(out)
        if shadow is not None:
            shadow.copy_(p)


def cast_(dst: torch.Tensor, src: torch.Tensor) -> None:
    """dst = src between fp32 and bf16 (same length, multiple of 4 on GPU)."""
    if dst.is_cuda and dst.numel() % 4 == 0:
        if src.dtype == torch.float32 and dst.dtype == torch.bfloat16:
            native().cast_f32_bf16(src.data_ptr(), dst.data_ptr(), dst.numel(), stream_handle())
            return
        if src.dtype == torch.bfloat16 and dst.dtype == torch.float32:
            native().cast_bf16_f32(src.data_ptr(), dst.data_ptr(), dst.numel(), stream_handle())
            return
    dst.copy_(src)


def add_(y: torch.Tensor, x: torch.Tensor) -> None:
    if y.is_cuda:
        native().add_inplace(y.data_ptr(), x.data_ptr(), y.numel(), stream_handle())
    else:
        y.add_(x)


def fill_(x: torch.Tensor, value: float, slot_value: float | None = None, slot_index: int = SLOT) -> None:
    if x.is_cuda and x.dtype == torch.float32 and x.numel() % 4 == 0:
        native().fill_f32(x.data_ptr(), float(value), x.numel(),
                          -1 if slot_value is None else int(slot_index), float(slot_value or 0.0), stream_handle())
        return
    x.fill_(value)
    if slot_value is not None:
        x.view(-1)[slot_index] = slot_value
