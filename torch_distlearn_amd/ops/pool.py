"""Channels-last max pooling on the HIP kernels of csrc/kernels/pool_nhwc.hip
(the ResNet-50 stem's 3x3/2 pool): argmax kept as one byte per output
element, gather-based backward (no atomics, no zero fill)."""
from __future__ import annotations

import torch

from .._native import native, stream_handle


def supported(x: torch.Tensor) -> bool:
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last))


class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k: int, s: int, p: int):
        N, C, H, W = x.shape
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        y = torch.empty((N, C, Ho, Wo), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        idx = torch.empty((N, Ho, Wo, C), dtype=torch.uint8, device=x.device)
        # x may be a deferred BN + ReLU output (ops/bn_nhwc.py defer_pool): pool its
        # input with the BN applied on load (csrc pool_nhwc.hip PoolBn)
        pb = getattr(x, "_dl_pool_bn", None)
        kw, src = {}, x
        if pb is not None:
            del x._dl_pool_bn
            xin, acc, w, b, save, rm, rv, eps, mom = pb[1]
            src = xin
            kw = dict(bn_acc=acc.data_ptr(), bn_w=w.data_ptr(), bn_b=b.data_ptr(), bn_save=save.data_ptr(),
                      bn_rm=rm.data_ptr() if rm is not None else 0, bn_rv=rv.data_ptr() if rv is not None else 0,
                      bn_eps=float(eps), bn_momentum=float(mom))
        native().maxpool_nhwc_fwd(src.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, k, s, p, stream_handle(),
                                  **kw)
        # ... and its backward then runs the BN's backward too (maxpool_bn_bwd)
        ctx.bn_link = getattr(x, "_dl_pool_bwd", None) if pb is not None else None
        if ctx.bn_link is not None:
            del x._dl_pool_bwd
        ctx.backwards = 0
        ctx.save_for_backward(idx)
        ctx.geom = (N, C, H, W, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, k, s, p = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        link = ctx.bn_link
        ctx.backwards += 1
        if link is not None and "fwd" in link:
            # dx = the input gradient of the BN + ReLU before the pool (its sums and
            # dgamma / dbeta too): that BN's backward passes it through
            xb, save, w, b, acc4, grads = link["fwd"]
            accb = acc4[2 * C:]
            if ctx.backwards > 1:
                accb.zero_()
            dw, db = (grads[0], grads[1]) if grads is not None else (
                torch.empty(C, device=dy.device), torch.empty(C, device=dy.device))
            native().maxpool_bn_bwd(dy.data_ptr(), idx.data_ptr(), xb.data_ptr(), save.data_ptr(), w.data_ptr(),
                                    b.data_ptr(), accb.data_ptr(), dx.data_ptr(), dw.data_ptr(), db.data_ptr(), N, H,
                                    W, C, stream_handle())
            link["fused"] = True
            link["dwdb"] = (dw, db)
            return dx, None, None, None
        native().maxpool_nhwc_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, C, k, s, p, stream_handle())
        return dx, None, None, None


def max_pool2d_nhwc(x: torch.Tensor, k: int, s: int, p: int) -> torch.Tensor:
    if not supported(x):
        raise ValueError("max_pool2d_nhwc: needs a channels-last bf16 CUDA tensor with C % 8 == 0")
    if getattr(x, "_dl_pool_bn", None) is not None and not (k == 3 and s == 2 and p == 1 and 256 % (x.shape[1] // 8) == 0):
        from .bn_nhwc import materialize

        materialize(x)  # this window cannot apply the deferred BN on load
    return _MaxPool.apply(x, k, s, p)
