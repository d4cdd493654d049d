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
  folded in), the bias gradient (fp32 atomics into the flat gradient);
* the backward GEMMs run here too (the loss is the graph's root, so its
  gradient is 1): d(pooled) = dlogits W (``conv_fwd``), the weight gradient
  dlogits^T f (``conv_wgrad`` + ``head_wgrad_reduce`` x 49 into the flat
  gradient), and ``head_broadcast`` expands d(pooled) over the 7x7 positions.

``backward`` only hands the stashed input gradient to autograd: the loss is
the root of the training graph (``loss.backward()``, d loss = 1).
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
            ctx.dh = None
            return loss[0], logp
        gw, gb, ready = bind
        loss_b = torch.empty(B, device=dev)
        dl = torch.empty(B, NCp, dtype=BF16, device=dev)
        C.head_softmax_nll(slab.data_ptr(), splits, B, ncls, NCp, fc_b.data_ptr(), labels.data_ptr(), logp.data_ptr(),
                           loss_b.data_ptr(), dl.data_ptr(), 1.0 / (B * HW), gb.data_ptr(), loss.data_ptr(), s)
        # d(pooled) = dl W  ([B, NCp] x [NCp, C]: a 1x1 conv whose weight is W^T)
        df = torch.empty(B, Cc, dtype=BF16, device=dev)
        dt, ds = _fwd_plan(B, Cc, NCp)
        dslab = torch.empty(ds * B * Cc, device=dev) if ds > 1 else None
        C.conv_fwd(dl.data_ptr(), wbt.data_ptr(), df.data_ptr(), 0, 0 if dslab is None else dslab.data_ptr(), B, 1, 1,
                   NCp, Cc, 1, dt, ds, s)
        dh = torch.empty_like(h, memory_format=torch.channels_last)
        C.head_broadcast(df.data_ptr(), dh.data_ptr(), B, HW, Cc, s)
        # dW = dl^T f ([NCp, B] x [B, C]) -> x HW (dl carries 1/(B*HW)) into the flat gradient
        from .conv import _wgrad_plan

        wt_tile, wsplits = _wgrad_plan(NCp, Cc, B)
        ws = torch.empty(wsplits * NCp * Cc, device=dev)
        C.conv_wgrad(dl.data_ptr(), f.data_ptr(), ws.data_ptr(), B, 1, 1, Cc, NCp, 1, wsplits, Cc, wt_tile, 0, s)
        C.head_wgrad_reduce(ws.data_ptr(), gw.data_ptr(), wsplits, ncls, NCp, Cc, float(HW), s)
        ready()
        ctx.dh = dh
        return loss[0], logp

    @staticmethod
    def backward(ctx, dloss, dlogp):
        dh = ctx.dh
        ctx.dh = None
        # the loss is the root of the training graph (d loss = 1): every gradient
        # was computed in forward for exactly that root
        return dh, None, None, None, None
