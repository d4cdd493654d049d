"""ResNet-50 classifier head on the MFMA kernels: spatial mean + Linear(2048,
1000) + LogSoftMax + ClassNLLCriterion (mean), forward AND backward in one
autograd node (BASELINE config 5; the reference's Linear + LogSoftMax + NLL are
cunn modules, examples/cifar10.lua:132-143).

Forward (training, labels given):

* ``head_weight_prep``: bf16 copies of the fp32 classifier weight, padded to
  1024 rows (W) and transposed (W^T) -- one launch;
* ``head_pool``: f = bf16(mean over the 7x7 positions) [B, 2048];
* logits on the MFMA GEMM kernel as a split-K 1x1 conv (``conv_fwd``, keep-
  slabs bit: fp32 partial slabs, no bf16 logits);
* ``head_softmax_nll``: sums the slabs + bias in fp32, log-softmax, per-sample
  loss and its mean, dlogits (bf16, scaled by 1/(B*49): the mean's backward
  folded in), the bias gradient (fp32 atomics into a per-step buffer);
* backward (``d loss`` from autograd, 1 when the loss is the graph's root):
  dlogits and the bias gradient are scaled by ``d loss`` on the device (no
  host sync), then d(pooled) = dlogits W (``conv_fwd``), the weight gradient
  dlogits^T f (``conv_wgrad`` + ``head_wgrad_reduce`` x 49, accumulated into
  the flat gradient) and ``head_broadcast`` expands d(pooled) over the 7x7
  positions; the bucket is reported ready.

Contract: the loss output may be scaled or combined with other terms (its
gradient is honoured); the log-probability output is for metrics only -- a
loss built on it raises in backward instead of training with a wrong
gradient.  One backward per forward.  Labels must be int64 on the device; an
out-of-range label makes that sample's loss (and the mean) NaN instead of
reading past the logits.
"""
from __future__ import annotations

import torch

from .._native import native, stream_handle

BF16 = torch.bfloat16


def head_supported(h: torch.Tensor, ncls: int) -> bool:
    n, c, hh, ww = h.shape
    return (h.is_cuda and h.dtype == BF16 and h.is_contiguous(memory_format=torch.channels_last) and c % 128 == 0
            and ncls <= 1024 and n >= 1)


def _ncp(ncls: int) -> int:
    return (ncls + 127) // 128 * 128


class ResNetHeadNLL(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, fc_w, fc_b, labels, bind):
        """h: channels-last bf16 [B, C, H, W]; returns (mean loss, log-probs
        [B, ncls] fp32).  ``bind``: (weight grad view, bias grad view, ready)
        or None (eval: no gradients)."""
        C = native()
        s = stream_handle()
        B, Cc, H, W = h.shape
        HW = H * W
        ncls = fc_w.shape[0]
        NCp = _ncp(ncls)
        dev = h.device
        wb = torch.empty(NCp, Cc, dtype=BF16, device=dev)
        wbt = torch.empty(Cc, NCp, dtype=BF16, device=dev)
        C.head_weight_prep(fc_w.data_ptr(), wb.data_ptr(), wbt.data_ptr(), ncls, NCp, Cc, s)
        f = torch.empty(B, Cc, dtype=BF16, device=dev)
        loss = torch.empty(4, device=dev)
        C.head_pool(h.data_ptr(), f.data_ptr(), B, HW, Cc, loss.data_ptr(), s)
        from .conv import _fwd_plan

        tile, splits = _fwd_plan(B, NCp, Cc)
        splits = max(splits, 2)  # the fp32 slabs ARE the logits (never rounded to bf16)
        slab = torch.empty(splits * B * NCp, device=dev)
        C.conv_fwd(f.data_ptr(), wb.data_ptr(), f.data_ptr(), 0, slab.data_ptr(), B, 1, 1, Cc, NCp, 1,
                   tile | (1 << 20), splits, s)
        logp = torch.empty(B, ncls, device=dev)
        train = labels is not None and bind is not None
        if not train:
            C.head_softmax_nll(slab.data_ptr(), splits, B, ncls, NCp, fc_b.data_ptr(), 0, logp.data_ptr(), 0, 0, 1.0,
                               0, 0, s)
            ctx.saved = None
            return loss[0], logp
        if labels.dtype != torch.int64 or labels.device != h.device or labels.numel() != B:
            raise ValueError("ResNetHeadNLL: labels must be int64 [B] on the activations' device")
        loss_b = torch.empty(B, device=dev)
        dl = torch.empty(B, NCp, dtype=BF16, device=dev)
        db = torch.zeros(ncls, device=dev)  # this step's bias gradient, scaled by d loss in backward
        C.head_softmax_nll(slab.data_ptr(), splits, B, ncls, NCp, fc_b.data_ptr(), labels.data_ptr(), logp.data_ptr(),
                           loss_b.data_ptr(), dl.data_ptr(), 1.0 / (B * HW), db.data_ptr(), loss.data_ptr(), s)
        ctx.set_materialize_grads(False)
        ctx.saved = (f, dl, db, wbt, bind, (B, Cc, H, W, ncls, NCp))
        return loss[0], logp

    @staticmethod
    def backward(ctx, dloss, dlogp):
        if dlogp is not None:
            raise RuntimeError("ResNetHeadNLL: the log-probability output is not differentiable (use the loss output)")
        if getattr(ctx, "saved", None) is None:
            raise RuntimeError("ResNetHeadNLL: backward ran twice (or on an eval forward)")
        f, dl, db, wbt, (gw, gb, ready), (B, Cc, H, W, ncls, NCp) = ctx.saved
        ctx.saved = None
        if dloss is None:
            return None, None, None, None, None
        C = native()
        s = stream_handle()
        dev = f.device
        HW = H * W
        dl.mul_(dloss)              # d loss (1.0 at the root: exact)
        gb.add_(db * dloss)
        # d(pooled) = dl W  ([B, NCp] x [NCp, C]: a 1x1 conv whose weight is W^T)
        from .conv import _fwd_plan, _wgrad_plan

        df = torch.empty(B, Cc, dtype=BF16, device=dev)
        dt, ds = _fwd_plan(B, Cc, NCp)
        dslab = torch.empty(ds * B * Cc, device=dev) if ds > 1 else None
        C.conv_fwd(dl.data_ptr(), wbt.data_ptr(), df.data_ptr(), 0, 0 if dslab is None else dslab.data_ptr(), B, 1, 1,
                   NCp, Cc, 1, dt, ds, s)
        dh = torch.empty(B, Cc, H, W, dtype=BF16, device=dev, memory_format=torch.channels_last)
        C.head_broadcast(df.data_ptr(), dh.data_ptr(), B, HW, Cc, s)
        # dW = dl^T f ([NCp, B] x [B, C]) -> x HW (dl carries 1/(B*HW)) accumulated into the flat gradient
        wt_tile, wsplits = _wgrad_plan(NCp, Cc, B)
        ws = torch.empty(wsplits * NCp * Cc, device=dev)
        C.conv_wgrad(dl.data_ptr(), f.data_ptr(), ws.data_ptr(), B, 1, 1, Cc, NCp, 1, wsplits, Cc, wt_tile, 0, s)
        C.head_wgrad_reduce(ws.data_ptr(), gw.data_ptr(), wsplits, ncls, NCp, Cc, float(HW), s)
        ready()
        return dh, None, None, None, None
