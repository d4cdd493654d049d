"""ResNet-50 (ImageNet shape, 25.6M parameters) -- BASELINE.json config 5:
"ResNet-50 ImageNet-shape synthetic AllReduceSGD bf16 (bucket fusion / xGMI
bandwidth stress)".  Not a model of the reference; it exists to exercise the
bucketed gradient all-reduce with a 102 MB fp32 gradient (~25 MB
buckets, >= 4 per step).

Compute path: channels-last bf16 with fp32 master weights in the flat
buffer.  Every convolution -- the stride-1 1x1 GEMMs and 3x3s, the stride-2
1x1 / 3x3 convolutions and the 7x7 stem -- runs on the hand-written MFMA
kernels (ops/conv.py), the classifier on the fused head kernels (ops/head.py);
BatchNorm(+ReLU, +residual) runs on the channels-last HIP kernels with fp32
statistics (ops/bn_nhwc.py).  MIOpen is only an A/B option (``_CONV_MODE``,
``_STRIDED_HIP``) and the eval-mode fallback of modules that were never bound
to a trainer's flat buffers.  Parameters are
registered in forward order, so :meth:`FlatParams.buckets` (reverse order)
puts the classifier and last stage in the first bucket to be reduced.
"""
from __future__ import annotations

from typing import List, Optional

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

# BatchNorm path: "mixed" feeds the bf16 activation straight to
# the BN kernel, which keeps fp32 statistics / affine parameters internally;
# "fp32" materialises an fp32 copy of every activation first (one extra full
# read + write of each BN input and output in HBM); "hip" runs training BN
# fused with its ReLU / residual add on the channels-last HIP kernels
# (ops/bn_nhwc.py, csrc/kernels/bn_nhwc.hip; default: 43.7 -> 35.5 ms/step).
_BN_MODE = os.environ.get("DISTLEARN_RESNET_BN", "hip")
# eval-mode BatchNorm (predict) on the same HIP apply kernel from the running
# statistics (False: F.batch_norm on an fp32 copy, the tests' reference)
_BN_EVAL_HIP = True


class _BN(nn.Module):
    def __init__(self, c: int, zero: bool = False):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(c) if zero else torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))
        self.bind = None  # (weight grad view, bias grad view, ready) -- ResNet50.attach_flat
        self.acc = None  # this step's zeroed fp32 [4C] slice of the model's statistics arena
        self.pad_bufs = {}  # persistent zero-bordered output / input-gradient buffers (ops/bn_nhwc.py padded_buffer)

    def forward(self, x):
        if _BN_MODE == "mixed" and x.is_cuda:
            return F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias, self.training, 0.1,
                                1e-5)
        y = F.batch_norm(x.float(), self.running_mean, self.running_var, self.weight, self.bias, self.training, 0.1,
                         1e-5)
        return y.to(x.dtype)

    def hip_ok(self, x, residual=None) -> bool:
        if not (_BN_MODE == "hip" and self.training and x.is_cuda):
            return False
        from ..ops.bn_nhwc import supported

        return supported(x) and self.weight.dtype == torch.float32 and (
            residual is None or (residual.dtype == x.dtype and residual.shape == x.shape))

    def hip_eval_ok(self, x, residual=None) -> bool:
        if not (_BN_MODE == "hip" and not self.training and x.is_cuda and _BN_EVAL_HIP):
            return False
        if torch.is_grad_enabled() and (x.requires_grad or self.weight.requires_grad):
            return False  # differentiable eval forward: the torch op
        from ..ops.bn_nhwc import supported

        return supported(x) and self.weight.dtype == torch.float32 and (
            residual is None or (residual.dtype == x.dtype and residual.shape == x.shape))

    def act(self, x, relu: bool = True, residual=None, acc=None, res_sink=None, have_stats: bool = False,
            out_pad: int = 0, dx_pad: int = 0, defer: bool = False, defer_pool: bool = False):
        """act(BN(x) [+ residual]); one fused HIP kernel pair in "hip" mode
        (``acc`` with ``have_stats``: statistics already accumulated by the
        producing conv; else the step's zeroed arena slice, if any;
        ``out_pad`` / ``dx_pad``: zero-bordered output / input gradient;
        ``defer``: no ReLU / residual -- the output is a handle the consuming
        BN + residual + ReLU applies on load, ops/bn_nhwc.py defer_apply)."""
        if residual is not None and getattr(residual, "_dl_res_bn", None) is not None and not self.hip_ok(x, residual):
            from ..ops.bn_nhwc import materialize

            materialize(residual)  # this BN cannot apply the deferred residual BN on load
        if self.hip_eval_ok(x, residual):  # eval / predict: the same HIP kernel from the running statistics
            from ..ops.bn_nhwc import bn_act_eval

            return bn_act_eval(x, self.weight, self.bias, self.running_mean, self.running_var, residual, relu,
                               out_pad=out_pad)
        if self.hip_ok(x, residual):
            from ..ops.bn_nhwc import bn_act

            if acc is None:
                acc, have_stats = self.acc, False
            return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, residual, relu, acc=acc,
                          grads=self.bind, res_sink=res_sink, have_stats=have_stats if acc is not None else None,
                          out_pad=out_pad, dx_pad=dx_pad,
                          defer_apply=defer and not relu and residual is None and have_stats and acc is not None,
                          defer_pool=defer_pool and relu and residual is None and have_stats and acc is not None
                          and not out_pad, pad_key=self.pad_bufs if _PAD_PERSIST else None)
        y = self(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y


# Convolution path once the trainer has bound the flat buffers (attach_flat):
# "hip" = every convolution on the hand-written MFMA kernels (stride-1 1x1 / 3x3,
# and with _STRIDED_HIP the strided ones and the stem), all reading the bf16 shadow
# weights (ops/conv.py); "miopen" = every convolution on MIOpen (A/B baseline).
_CONV_MODE = os.environ.get("DISTLEARN_RESNET_CONV", "hip")
# BatchNorm statistics from the 1x1 GEMM epilogue (skips the BN statistics pass)
_FUSE_STATS = True
# residual gradient added in the c1 dgrad epilogue (ops/conv.py conv_fwd_add).  With
# the first epilogue (per-element 2-byte addend loads) the dgrad took 308 us instead
# of 74 us (profiles/r2_resnet50_kernels_fuse_res.txt); the transposed epilogue loads
# the addend 16 bytes at a time and the fusion now wins: 30.33 -> 29.68 ms/step.
_FUSE_RES = True
# stride-1 3x3 convolutions on the hand-written implicit-GEMM kernels (ops/conv.py
# Conv3x3) for feature maps of at most this size (0 = off: MIOpen for all 3x3).
# The 56x56 stage joined once the wgrad ran on the XCD-aware grid with one round
# of 512 64x64 workgroups (161 vs MIOpen's 167 us; forward 88 vs 117 us:
# profiles/r2_conv3x3_sweep_v2.jsonl); end to end 25.93 vs 25.94 ms/step with
# the stage on MIOpen (profiles/r2_resnet_conv3_56_ab.txt).
_CONV3_MAX_HW = 56
# channels-last copies of the KxK shadows (the HIP 3x3 / stem kernels' KRSC operand and
# MIOpen's layout in the A/B mode), one launch per step (ops/conv.py)
_CL_WEIGHTS = True
# stem max-pool on the HIP gather-backward kernels (ops/pool.py)
_POOL_HIP = True
# stride-2 1x1 / 3x3 convolutions and the stem on the generalised MFMA kernels
# (ops/conv.py Conv1x1S2 / Conv3x3S2 / StemConv; False = MIOpen, A/B)
_STRIDED_HIP = True
# classifier (mean + Linear + LogSoftMax + NLL, forward and backward) in one node on the
# MFMA kernels (ops/head.py; 0 = torch mean / hipBLAS linear / torch log-softmax)
_HEAD_HIP = True
# (Rejected and removed in round 6: the BatchNorm backward sums in the epilogue
# of the dgrad that produces the BN's output gradient -- the reduce pass goes,
# -1.64 ms/step, but every fused epilogue re-reads the BN input, +2.0 ms,
# profiles/r5_resnet_bn_dgrad_ab.txt; b2's BN + ReLU applied by c3's GEMM on
# load, 25.43 vs 24.64 ms/step, profiles/r4_resnet_bn_on_load_ab.txt.)
# the downsample branch's BatchNorm applied on load by the block's b3 apply (csrc
# bn_nhwc.hip ResBn): b3 reads the downsample conv's output and applies that BN
# itself, so the downsample BN's apply launch and the write + read of its output
# go (4 per step, ~0.28 ms at batch 256)
_DEFER_DOWN_BN = True
# the stem BatchNorm + ReLU applied on load by the stem max-pool (csrc pool_nhwc.hip
# PoolBn): the apply launch and the write + read of its 112x112x64 output go
_DEFER_STEM_BN = True
# the zero-bordered BN outputs / input gradients of the 3x3 convs in buffers that
# persist per BatchNorm (border zeroed once, not by a zero_border launch per use):
# 23.66-23.72 vs 23.72-23.92 ms/step (profiles/r5_resnet_pad_persist_ab.txt).  (The
# first-loss mismatch seen with it was the head's atomic loss sum, which flips the
# last bit of the mean run to run with or without it.)
_PAD_PERSIST = True


class _Conv(nn.Module):
    def __init__(self, cin, cout, k, stride=1, g=None):
        super().__init__()
        fan = cin * k * k
        self.weight = nn.Parameter(torch.randn(cout, cin, k, k, generator=g) * (2.0 / fan) ** 0.5)
        self.stride, self.pad, self.k = stride, k // 2, k
        self.bind = None  # ops.conv.ShadowBinding (set by ResNet50.attach_flat)

    def hip_gemm(self, x) -> bool:
        """Stride-1 1x1 convolution on the hand-written MFMA GEMM kernels."""
        if self.bind is None or not x.is_cuda or x.dtype != torch.bfloat16:
            return False
        from ..ops.conv import conv1x1_supported

        return _CONV_MODE == "hip" and self.k == 1 and self.stride == 1 and conv1x1_supported(x, self.weight.shape[0])

    def hip_strided(self, x, shape=None) -> bool:
        """The stride-2 1x1 / 3x3 convolutions and the 7x7 stem on the
        generalised MFMA kernels (ops/conv.py Conv1x1S2 / Conv3x3S2 / StemConv)."""
        shape = tuple(x.shape) if shape is None else shape
        if (self.bind is None or not x.is_cuda or x.dtype != torch.bfloat16 or _CONV_MODE != "hip"
                or not _STRIDED_HIP or self.stride != 2):
            return False
        n, cin, h, w = shape
        cout = self.weight.shape[0]
        pow2 = lambda v: v >= 64 and (v & (v - 1)) == 0  # noqa: E731
        if self.k == 7:
            return cin == 3 and cout % 64 == 0
        if self.k == 3:
            return (self.bind.wcl is not None and pow2(cin) and pow2(cout) and h % 2 == 0 and w % 2 == 0
                    and n * (h + 2) * (w + 2) * max(cin, cout) < (1 << 31))
        return self.k == 1 and pow2(cin) and pow2(cout) and n * h * w * max(cin, cout) < (1 << 31)

    def hip_3x3(self, x, shape=None) -> bool:
        """Stride-1 3x3 convolution on the hand-written kernels (needs the
        channels-last shadow, ChannelsLastWeights) for an input like ``x``
        (device / dtype) of ``shape`` (default x.shape)."""
        shape = tuple(x.shape) if shape is None else shape
        if (self.bind is None or self.bind.wcl is None or self.k != 3 or self.stride != 1 or not x.is_cuda
                or x.dtype != torch.bfloat16 or _CONV_MODE != "hip" or shape[2] > _CONV3_MAX_HW):
            return False
        from ..ops.conv import conv3x3_supported

        return conv3x3_supported(shape, self.weight.shape[0])

    def forward(self, x, stats=None, res_link=None, dx_sink=None):
        """``stats``: optional fp32 [2*Cout] that receives the output's
        per-channel sum / sum of squares (HIP GEMM path only); ``res_link``:
        a dict through which another branch hands over its gradient of the
        same input (added in the dgrad epilogue); ``dx_sink``: the dict that
        receives THIS conv's input gradient instead of autograd."""
        b = self.bind
        if b is None or not x.is_cuda or x.dtype != torch.bfloat16:
            return F.conv2d(x, self.weight.to(x.dtype), None, self.stride, self.pad)
        from ..ops.conv import Conv1x1, ShadowConv

        # the same HIP kernels in training and in eval / predict (no-grad) mode
        grad = torch.is_grad_enabled()
        if self.hip_gemm(x):
            return Conv1x1.apply(x, self.weight, b, stats, res_link if grad else None, dx_sink if grad else None)
        if self.hip_3x3(x) and dx_sink is None:
            from ..ops.conv import Conv3x3

            return Conv3x3.apply(x, self.weight, b, stats)
        if self.hip_strided(x):
            from ..ops.conv import Conv1x1S2, Conv3x3S2, StemConv

            if self.k == 7:
                return StemConv.apply(x, self.weight, b, stats)
            if self.k == 3 and dx_sink is None:
                return Conv3x3S2.apply(x, self.weight, b, stats)
            if self.k == 1:
                return Conv1x1S2.apply(x, self.weight, b, stats, dx_sink if torch.is_grad_enabled() else None)
        if not torch.is_grad_enabled():
            w = b.wcl if b.wcl is not None else b.w16.view(self.weight.shape)
            return F.conv2d(x, w, None, self.stride, self.pad)
        return ShadowConv.apply(x, self.weight, b, self.stride, self.pad, dx_sink)


def _conv_bn(conv: _Conv, bn: "_BN", x, relu: bool = True, residual=None, link=None, res_sink=None, dx_sink=None,
             out_pad: int = 0, dx_pad: int = 0, defer: bool = False, defer_pool: bool = False):
    """bn.act(conv(x)) with the BatchNorm statistics produced by the conv's
    epilogue when both run on the HIP kernels (one full read of the conv
    output fewer per BatchNorm).  ``out_pad`` / ``dx_pad``: the BatchNorm writes
    its output / input gradient zero-bordered (for a Conv3x3 neighbour).
    ``defer`` / ``defer_pool``: the BN is applied on load by its consumer (the
    block's b3, the stem max-pool)."""
    kw = {"res_link": link, "dx_sink": dx_sink} if conv.bind is not None else {}
    pads = {"out_pad": out_pad, "dx_pad": dx_pad}
    if _FUSE_STATS and (conv.hip_gemm(x) or conv.hip_3x3(x) or conv.hip_strided(x)) and _BN_MODE == "hip" \
            and bn.training:
        from .._native import native

        if native().reduce_atomic() == 0:  # partial-row statistics (deterministic)
            cout = conv.weight.shape[0]
            acc = bn.acc if bn.acc is not None else torch.zeros(4 * cout, device=x.device)
            y = conv(x, stats=acc[:2 * cout], **kw)
            if bn.hip_ok(y, residual):
                return bn.act(y, relu, residual, acc=acc, res_sink=res_sink, have_stats=True, defer=defer,
                              defer_pool=defer_pool, **pads)
            return bn.act(y, relu, residual)
    return bn.act(conv(x, **kw), relu, residual, res_sink=res_sink, **pads)


class _Bottleneck(nn.Module):
    def __init__(self, cin, width, stride, g):
        super().__init__()
        cout = width * 4
        self.c1, self.b1 = _Conv(cin, width, 1, 1, g), _BN(width)
        self.c2, self.b2 = _Conv(width, width, 3, stride, g), _BN(width)
        self.c3, self.b3 = _Conv(width, cout, 1, 1, g), _BN(cout, zero=True)
        self.down = None
        if stride != 1 or cin != cout:
            self.down = nn.ModuleList([_Conv(cin, cout, 1, stride, g), _BN(cout)])

    def forward(self, x):
        # x feeds c1 (HIP GEMM) and a second branch: the identity residual (its
        # BatchNorm b3 hands the gradient of x over) or the downsample conv (hands
        # its dgrad over); c1's dgrad epilogue adds it -- no separate gradient sum.
        # Autograd normally runs the second branch's backward first (its nodes are
        # younger); if it does not, Conv1x1 marks the link done and the other branch
        # returns its gradient through autograd, which sums the two.
        link = {} if (_FUSE_RES and torch.is_grad_enabled() and self.c1.hip_gemm(x)
                      and (self.down is None or self.down[0].bind is not None)) else None
        # a stride-1 3x3 c2 on the HIP kernels reads b1's output and b2's input
        # gradient zero-bordered, written so by the BatchNorm kernels themselves
        n, _, h, w = x.shape  # c1 is 1x1 stride 1: c2's input is [n, width, h, w]
        c2in = (n, self.c2.weight.shape[1], h, w)
        pad = 1 if (self.c2.hip_3x3(x, c2in) or (self.c2.k == 3 and self.c2.hip_strided(x, c2in))) else 0
        y = _conv_bn(self.c1, self.b1, x, link=link, out_pad=pad)
        y = _conv_bn(self.c2, self.b2, y, dx_pad=pad)
        if self.down is None:
            return _conv_bn(self.c3, self.b3, y, residual=x, res_sink=link)
        # (the downsample BN's apply deferred into b3's: csrc ResBn)
        s = _conv_bn(self.down[0], self.down[1], x, relu=False, dx_sink=link, defer=_DEFER_DOWN_BN)
        return _conv_bn(self.c3, self.b3, y, residual=s)


class ResNet50(nn.Module):
    def __init__(self, num_classes: int = 1000, layers: List[int] = (3, 4, 6, 3), seed: Optional[int] = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        self.stem, self.stem_bn = _Conv(3, 64, 7, 2, g), _BN(64)
        blocks, cin = [], 64
        for i, n in enumerate(layers):
            width = 64 << i
            for j in range(n):
                blocks.append(_Bottleneck(cin, width, 2 if (j == 0 and i > 0) else 1, g))
                cin = width * 4
        self.blocks = nn.ModuleList(blocks)
        self.fc_w = nn.Parameter(torch.randn(num_classes, cin, generator=g) * (1.0 / cin) ** 0.5)
        self.fc_b = nn.Parameter(torch.zeros(num_classes))
        self._fc_bind = None  # (fc_w grad view, fc_b grad view, ready) -- attach_flat

    def trunk(self, x: torch.Tensor, compute_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """Stem + max-pool + the 16 bottlenecks: [B, 2048, 7, 7] features."""
        if x.dim() == 4 and x.shape[-1] == 3:
            x = x.permute(0, 3, 1, 2)
        cd = compute_dtype or x.dtype
        h = x.to(cd)
        if h.is_cuda:
            h = h.contiguous(memory_format=torch.channels_last)
        self._begin_step(h)
        # (with the HIP pool, the stem BN + ReLU is applied by the pool on load: PoolBn)
        h = _conv_bn(self.stem, self.stem_bn, h, defer_pool=_POOL_HIP and _DEFER_STEM_BN)
        from ..ops.bn_nhwc import materialize
        from ..ops.pool import max_pool2d_nhwc, supported

        h = max_pool2d_nhwc(h, 3, 2, 1) if (_POOL_HIP and supported(h)) else F.max_pool2d(materialize(h), 3, 2, 1)
        for b in self.blocks:
            h = b(h)
        return h

    def _hip_head(self, h) -> bool:
        from ..ops.head import head_supported

        return _HEAD_HIP and _CONV_MODE == "hip" and head_supported(h, self.fc_w.shape[0])

    def forward(self, x: torch.Tensor, compute_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """x: NHWC [B, H, W, 3] (or NCHW); returns log-probabilities (fp32)."""
        h = self.trunk(x, compute_dtype)
        # the fused head node computes gradients only for the training loss
        # (forward_loss); a differentiable forward() keeps the torch classifier
        if self._hip_head(h) and not (torch.is_grad_enabled() and (h.requires_grad or self.fc_w.requires_grad)):
            from ..ops.head import ResNetHeadNLL

            return ResNetHeadNLL.apply(h, self.fc_w, self.fc_b, None, None)[1]
        # classifier in fp32 (2048 x 1000: negligible cost): bf16 logits of a
        # memorising synthetic run overflowed into NaN at lr 0.1
        h = h.float().mean((2, 3))
        return F.log_softmax(F.linear(h, self.fc_w, self.fc_b), dim=1)

    def forward_loss(self, x: torch.Tensor, y: torch.Tensor, compute_dtype: Optional[torch.dtype] = None):
        """(mean NLL loss, log-probabilities) of a training step with the
        classifier head fused into one node (ops/head.py: mean + Linear +
        LogSoftMax + NLL forward and backward on the MFMA kernels), or None
        when that path does not apply (the caller then uses forward + loss)."""
        if self._fc_bind is None or not torch.is_grad_enabled():
            return None
        h = self.trunk(x, compute_dtype)
        if not self._hip_head(h):
            logp = F.log_softmax(F.linear(h.float().mean((2, 3)), self.fc_w, self.fc_b), dim=1)
            return self.loss(logp, y), logp
        from ..ops.head import ResNetHeadNLL

        return ResNetHeadNLL.apply(h, self.fc_w, self.fc_b, y, self._fc_bind)

    def _begin_step(self, h) -> None:
        """Per training step: ONE zero fill for every BatchNorm's forward and
        backward statistics (53 x 2 fills of ~5 us before), and ONE launch that
        refreshes the transposed 1x1 shadows for the dgrads."""
        train = torch.is_grad_enabled() and h.is_cuda and self.training
        bns = self._bns if hasattr(self, "_bns") else [m for m in self.modules() if isinstance(m, _BN)]
        self._bns = bns
        if train and _BN_MODE == "hip" and h.dtype == torch.bfloat16:
            arena = torch.zeros(sum(4 * m.weight.numel() for m in bns), device=h.device)
            o = 0
            for m in bns:
                m.acc = arena[o:o + 4 * m.weight.numel()]
                o += 4 * m.weight.numel()
        else:
            for m in bns:
                m.acc = None
        if train and getattr(self, "_wt", None) is not None:
            self._wt.refresh()
        if getattr(self, "_wcl", None) is not None and h.is_cuda:
            self._wcl.refresh()  # also read by the no-grad (predict) path

    @staticmethod
    def loss(logp, target):
        return F.nll_loss(logp, target)

    def attach_flat(self, flat, ready=None) -> None:
        """Bind every convolution to the trainer's flat buffers: it then reads
        its bf16 shadow weight and writes its fp32 gradient into the flat
        gradient directly, reporting it with ``ready(leaf_index)`` (the
        bucketed all-reduce) -- ops/conv.py."""
        from ..ops.conv import ShadowBinding

        if flat.shadow is None or flat.grad is None:
            return
        index = {id(t): i for i, t in enumerate(flat.leaves)}
        w16, g32 = flat.shadow_views(), flat.views_of(flat.grad)
        gemm, spatial = [], []
        for m in self.modules():
            if isinstance(m, _Conv):
                i = index[id(m.weight)]
                m.bind = ShadowBinding(w16[i], g32[i], (lambda i=i: ready(i)) if ready else (lambda: None))
                if m.k == 1 and w16[i].is_cuda:  # stride 1 and 2: transposed shadow for the dgrad
                    gemm.append(m.bind)
                elif m.k > 1 and w16[i].is_cuda:
                    spatial.append((m.bind, tuple(m.weight.shape)))
            elif isinstance(m, _BN):
                # the HIP BatchNorm backward writes dgamma / dbeta straight into the flat gradient
                iw, ib = index[id(m.weight)], index[id(m.bias)]
                m.bind = (g32[iw], g32[ib], (lambda iw=iw, ib=ib: (ready(iw), ready(ib))) if ready else (lambda: None))
        iw, ib = index[id(self.fc_w)], index[id(self.fc_b)]
        self._fc_bind = (g32[iw], g32[ib], (lambda: (ready(iw), ready(ib))) if ready else (lambda: None))
        if gemm and _CONV_MODE == "hip":
            from ..ops.conv import WeightTransposes

            self._wt = WeightTransposes(gemm)
        if spatial and _CL_WEIGHTS:
            from ..ops.conv import ChannelsLastWeights

            self._wcl = ChannelsLastWeights([b for b, _ in spatial], [s for _, s in spatial])


def resnet50(num_classes: int = 1000, seed: Optional[int] = 0) -> ResNet50:
    return ResNet50(num_classes, seed=seed)
