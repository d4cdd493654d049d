"""Convolutions of the ResNet-50 path that read the FlatParams bf16 shadow and
write fp32 weight gradients straight into the flat gradient buffer.

Without this, every step casts every fp32 master weight to bf16 in the
forward (``weight.to(bf16)``) and casts + accumulates the bf16 weight gradient
back into the fp32 ``.grad`` in the backward: 376 elementwise kernels,
3.3 ms of a 35.5 ms ResNet-50 step (profiles/r1_resnet50_kernels.txt).  The
fused SGD kernel already keeps a bf16 shadow of every parameter
(csrc/kernels/flat_ops.hip ``sgd_kernel<.., kShadow>``), so:

* :class:`Conv1x1` -- stride-1 1x1 convolutions (2 of the 3 convolutions of
  every bottleneck) are plain NHWC GEMMs and run on the hand-written MFMA
  kernels of ``csrc/kernels/conv_igemm.hip`` (``M = N*H*W`` pixels as a batch
  of 1x1 images): forward ``y = x W^T`` (optionally emitting the following
  BatchNorm's per-channel sum / sum of squares: deterministic partial rows
  from its epilogue + a T x 2C column reduce, instead of the BatchNorm's own
  pass over the M x C output), dgrad
  ``dx = dy W`` (same kernel on the transposed shadow) and wgrad
  ``dW = dy^T x`` in fp32 (split-K partial slabs, reduced and added into the
  flat gradient by one kernel).
* :class:`Conv3x3` -- stride-1 3x3 convolutions on the same streaming MFMA
  kernel (zero-bordered NHWC inputs written by the BatchNorm kernels).
* :class:`Conv1x1S2` / :class:`Conv3x3S2` / :class:`StemConv` -- the strided
  convolutions and the 7x7 stem on the generalised MFMA kernels (conv_fwd_ex /
  conv_wgrad_ex).
* :class:`ShadowConv` -- MIOpen on the shadow weight, adding the weight gradient
  into the flat buffer: only the A/B baseline (``DISTLEARN_RESNET_CONV=miopen`` /
  ``DISTLEARN_RESNET_STRIDED=0``), not used by the default training step.

Both mark their weight's gradient ready for the bucketed all-reduce
themselves (the autograd graph gets no weight gradient, so the
post-accumulate-grad hook would never fire).

Reference parity: these are the ResNet-50 stress config of BASELINE.json
(config 5); the reference's own convolutions are cunn SpatialConvolutionMM
(examples/cifar10.lua:108-126).
"""
from __future__ import annotations


import torch
import torch.nn.functional as F

from .._native import native, stream_handle

BF16 = torch.bfloat16

class ShadowBinding:
    """What a conv module needs from the trainer: its bf16 shadow weight view,
    its fp32 gradient view, and a callback that reports the gradient ready.
    ``wt``: optional [Cin][Cout] bf16 transposed shadow of a 1x1 weight that
    :class:`WeightTransposes` refreshes once per step (the dgrad B operand)."""

    __slots__ = ("w16", "g32", "ready", "wt", "wcl")

    def __init__(self, w16: torch.Tensor, g32: torch.Tensor, ready):
        self.w16, self.g32, self.ready = w16, g32, ready
        self.wt = None
        self.wcl = None  # channels-last copy of a KxK shadow (ChannelsLastWeights), for MIOpen


class WeightTransposes:
    """The transposed bf16 shadows of many 1x1 conv weights, refreshed by ONE
    kernel launch per step (csrc transpose_many) instead of one transpose per
    conv in its backward.  ``refresh()`` must run after the optimizer step has
    written the shadow and before the first dgrad reads ``bind.wt`` -- the
    model calls it at the start of every training forward."""

    def __init__(self, binds):
        C = native()
        binds = list(binds)
        dev = binds[0].w16.device
        total = sum(b.w16.numel() for b in binds)
        self.arena = torch.empty(total, dtype=BF16, device=dev)
        rows, o, tiles = [], 0, 0
        for b in binds:
            cout = b.w16.shape[0]
            cin = b.w16.numel() // cout
            b.wt = self.arena[o:o + cout * cin].view(cin, cout)
            tc = (cin + 63) // 64
            rows.append([b.w16.data_ptr(), b.wt.data_ptr(), cout | (cin << 32), tiles | (tc << 32)])
            tiles += ((cout + 63) // 64) * tc
            o += cout * cin
        if C.transpose_entry_bytes() != 32:
            raise RuntimeError("transpose_many: unexpected entry layout")
        self.table = torch.tensor(rows, dtype=torch.int64).to(dev)
        self.n, self.tiles = len(binds), tiles

    def refresh(self):
        native().transpose_many(self.table.data_ptr(), self.n, self.tiles, stream_handle())


def _fwd_plan(M: int, N: int, K: int):
    from ..models.cifar_hip import _fwd_plan as plan

    return plan(M, N, K)


def _plan_1x1(M: int, N: int, K: int):
    """(packed tile id, splits) of an M x K x N 1x1-conv GEMM.  Measured on the
    ResNet-50 shapes (profiles/r2_gemm1x1_sweep.jsonl, scripts/bench_gemm1x1.py
    SWEEP=1): a 2-stage LDS ring (two workgroups per CU) beats the 3-stage
    default by up to 1.5x on the short-K GEMMs, and 4-wave workgroups win when
    K <= 128; only the N = 64, K >= 256 GEMMs keep 3 stages.  Round-5 re-sweep
    (profiles/r5_gemm1x1_sweep.jsonl): the K = 128, N = 512 GEMMs of the 28x28
    stage now run faster on 8 waves (72.8 vs 77.0 us fwd, 73.5 vs 78.3 dgrad)."""
    tile, splits = _fwd_plan(M, N, K)
    if splits > 1:
        return tile, splits
    tile = 0 if N % 128 == 0 else 2
    stages = 3 if (N == 64 and K >= 256) else 2
    waves = 4 if (K <= 64 or (K <= 128 and N < 512)) else 8
    return tile | (stages << 4) | (waves << 8), 1


def _wgrad_plan(cout: int, K: int, M: int):
    from ..models.cifar_hip import _wgrad_plan as plan

    return plan(cout, K, M, 0)


def conv1x1_supported(x: torch.Tensor, cout: int) -> bool:
    cin = x.shape[1]
    pow2 = lambda v: v >= 8 and (v & (v - 1)) == 0  # noqa: E731
    M = x.shape[0] * x.shape[2] * x.shape[3]
    return (x.is_cuda and x.dtype == BF16 and pow2(cin) and pow2(cout) and cout % 64 == 0 and cin % 64 == 0
            and M * max(cin, cout) < (1 << 31))


class ChannelsLastWeights:
    """Channels-last copies of the KxK conv shadows for the MIOpen convolutions,
    refreshed by ONE launch per step (csrc weights_to_cl).  The flat buffer
    keeps every weight in [Cout][Cin][K][K] order, and torch copied each one to
    channels-last inside every F.conv2d / convolution_backward call on a
    channels-last input (34 copy kernels per ResNet-50 step)."""

    def __init__(self, binds, shapes):
        C = native()
        if C.cl_entry_bytes() != 32:
            raise RuntimeError("weights_to_cl: unexpected entry layout")
        binds = list(binds)
        dev = binds[0].w16.device
        self.arena = torch.empty(sum(b.w16.numel() for b in binds), dtype=BF16, device=dev)
        rows, o = [], 0
        for b, (cout, cin, k, _) in zip(binds, shapes):
            n = cout * cin * k * k
            b.wcl = self.arena[o:o + n].as_strided((cout, cin, k, k), (k * k * cin, 1, k * cin, cin))
            rows.append([b.w16.data_ptr(), b.wcl.data_ptr(), cout | (cin << 32), k * k])
            o += n
        self.table = torch.tensor(rows, dtype=torch.int64).to(dev)
        self.n = len(binds)

    def refresh(self):
        native().weights_to_cl(self.table.data_ptr(), self.n, stream_handle())


class Conv1x1(torch.autograd.Function):
    """y = conv1x1(x, W) on the MFMA kernels; x channels-last bf16 [N, Cin, H, W]."""

    @staticmethod
    def forward(ctx, x, weight, bind: ShadowBinding, stats, res_link=None, dx_sink=None):
        C = native()
        ctx.res_link = res_link
        ctx.dx_sink = dx_sink
        if dx_sink is not None:
            dx_sink["expect"] = True  # dx goes to the sink's consumer, not to autograd
        x = x.contiguous(memory_format=torch.channels_last)
        N, cin, H, W = x.shape
        cout = weight.shape[0]
        M = N * H * W
        y = torch.empty((N, cout, H, W), dtype=BF16, device=x.device, memory_format=torch.channels_last)
        tile, splits = _plan_1x1(M, cout, cin)
        slab = torch.empty(splits * M * cout, device=x.device) if splits > 1 else None
        s = stream_handle()
        rows = None
        if stats is not None:
            # the epilogue's deterministic per-M-tile partial sums (reduction mode 0) ...
            if C.reduce_atomic() != 0:
                raise RuntimeError("Conv1x1 statistics need reduction mode 0 (partial rows)")
            nrows = C.conv_fwd_stat_rows(M, 1, 1, cin, cout, 1, tile, splits)
            rows = torch.empty(max(nrows, 400 if splits > 1 else 1), 2, cout, device=x.device)
        T = C.conv_fwd(x.data_ptr(), bind.w16.data_ptr(), y.data_ptr(), 0 if rows is None else rows.data_ptr(),
                       0 if slab is None else slab.data_ptr(), M, 1, 1, cin, cout, 1, tile, splits, s)
        if rows is not None:  # ... -> sum / sum of squares per channel for the BatchNorm
            C.bn_rows_reduce(rows.data_ptr(), T, cout, stats.data_ptr(), s)
        ctx.save_for_backward(x)
        ctx.bind = bind
        ctx.geom = (M, cin, cout)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        (x,) = ctx.saved_tensors
        bind = ctx.bind
        M, cin, cout = ctx.geom
        s = stream_handle()
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = None
        add = s2 = add_mask = None
        link = ctx.res_link
        if link is not None and link.get("expect") and ctx.needs_input_grad[0]:
            # the same input also fed another branch (the identity residual's
            # BatchNorm, ops/bn_nhwc.py res_sink, or the downsample conv's dgrad,
            # dx_sink) that parked its gradient here: dx = dy W + that gradient
            # (a stride-2 downsample parks its deferred dgrad instead: "s2")
            add = link.pop("g", None)
            s2 = link.pop("s2", None)
            gm = link.pop("gm", None)  # (dy, mask bits): the residual gradient still to be masked
            if gm is not None:
                add, add_mask = gm
            if add is None and s2 is None:
                # autograd ran this branch first (no ordering guarantee): the other
                # branch returns its gradient through autograd, which sums them
                link["done"] = True
            elif add is not None:
                add = add.contiguous(memory_format=torch.channels_last)
        if ctx.needs_input_grad[0]:
            wt = bind.wt
            if wt is None:
                wt = torch.empty(cin, cout, dtype=BF16, device=x.device)
                C.weight_flip_transpose(bind.w16.data_ptr(), wt.data_ptr(), cout, cin, 1, s)
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            tile, splits = _plan_1x1(M, cin, cout)
            if add is not None and splits == 1:
                C.conv_fwd_add(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), add.data_ptr(), M, 1, 1, cout, cin,
                               1, tile, s, 0 if add_mask is None else add_mask.data_ptr())
                add = None
            else:
                slab = torch.empty(splits * M * cin, device=x.device) if splits > 1 else None
                C.conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, 0 if slab is None else slab.data_ptr(), M,
                           1, 1, cout, cin, 1, tile, splits, s)
            if add is not None:
                if add_mask is not None:  # (split-K dgrad: the masked residual gradient the slow way)
                    from .bn_nhwc import unpack_mask_bits

                    add = add.masked_fill(~unpack_mask_bits(add_mask, add), 0)
                dx.add_(add)
            if s2 is not None:  # dx[:, ::2, ::2] += the stride-2 downsample's dgrad (in place)
                Conv1x1S2.deferred_dgrad(C, s2[0], s2[1], s2[2], dx, s)
        elif add is not None:
            if add_mask is not None:
                from .bn_nhwc import unpack_mask_bits

                add = add.masked_fill(~unpack_mask_bits(add_mask, add), 0)
            dx = add
        # fp32 weight gradient added into the flat buffer: split-K partials in plain
        # slabs + one reduce-add (atomic split-K adds were 1.3-2.3x slower on every
        # ResNet-50 shape: device-scope fp32 atomics from all 8 XCDs contend,
        # profiles/r2_gemm1x1_wgrad_slab.jsonl)
        tile, splits = _wgrad_plan(cout, cin, M)
        ws = torch.empty(splits * cout * cin, device=x.device)
        C.conv_wgrad(dy.data_ptr(), x.data_ptr(), ws.data_ptr(), M, 1, 1, cin, cout, 1, splits, cin, tile, 0, s)
        C.slab_reduce_add(ws.data_ptr(), bind.g32.data_ptr(), splits, cout, 1, cin, cin, s)
        bind.ready()
        if ctx.dx_sink is not None and dx is not None:
            ctx.dx_sink["g"] = dx
            dx = None
        return dx, None, None, None, None, None


PAD_COPIES = [0]  # Conv3x3 inputs / gradients that had to be padded by a copy (tests)


def _padded_base(t: torch.Tensor, pad: int):
    """(tensor to keep alive, pointer of the [N][H+2p][W+2p][C] zero-bordered
    buffer) for a [N, C, H, W] activation: ``t`` itself when it is the
    interior view made by ops.bn_nhwc.padded_empty, else a padded copy."""
    n, c, h, w = t.shape
    hp, wp = h + 2 * pad, w + 2 * pad
    if getattr(t, "_dl_pad", 0) == pad and t.stride() == (hp * wp * c, 1, wp * c, c):
        return t, t.data_ptr() - (pad * wp + pad) * c * t.element_size()
    PAD_COPIES[0] += 1
    tp = F.pad(t.permute(0, 2, 3, 1), (0, 0, pad, pad, pad, pad)).contiguous()
    return tp, tp.data_ptr()


def conv3x3_supported(shape, cout: int, is_cuda: bool = True, dtype=BF16) -> bool:
    """Whether Conv3x3 takes an input of ``shape`` [N, Cin, H, W]."""
    n, cin, h, w = shape
    pow2 = lambda v: v >= 64 and (v & (v - 1)) == 0  # noqa: E731
    return (is_cuda and dtype == BF16 and pow2(cin) and pow2(cout) and n * h * w < (1 << 24)
            and n * (h + 2) * (w + 2) * max(cin, cout) < (1 << 31))


def _plan_3x3(M: int, N: int, K: int):
    """Forward / dgrad plan of a 3x3 GEMM (packed tile id, splits): 2-stage
    ring, 8 waves, no split -- the best of a stage/wave/tile/split sweep on
    every ResNet-50 stride-1 3x3 shape (scripts/bench_conv3x3.py SWEEP=1,
    profiles/r2_conv3x3_sweep.jsonl): 71-88 us vs MIOpen's 74-119 us forward.
    The 64-channel GEMMs (the 56x56 stage) run 4 waves since round 5: 93.8 vs
    114.4 us with 8 (profiles/r5_conv3x3_sweep.jsonl)."""
    tile = 0 if N % 128 == 0 else 2
    waves = 4 if (N == 64 and _W4_C64) else 8
    return tile | (2 << 4) | (waves << 8), 1


_W4_C64 = True  # (r5_conv3x3_sweep.jsonl)


def _wgrad_plan_3x3(cout: int, K: int, M: int):
    """Weight-gradient plan (tile, splits) of a 3x3 conv: about one round of
    workgroups, two when the tiles alone nearly fill the chip (same sweep).
    64x64 tiles (Cout = 64, the 56x56 stage) run two workgroups per CU, so one
    round is 512 of them: 56 splits, 161 us vs 28 splits' ~177 and MIOpen's
    167 (profiles/r2_conv3x3_sweep_v2.jsonl)."""
    tile = 2 if cout % 128 == 0 else 1
    bm, bn = (128, 128) if tile == 2 else (64, 64)
    tiles = (cout // bm) * ((K + bn - 1) // bn)
    slots = 512 if (tile == 1 or tiles > 64) else 256
    splits = max(1, slots // tiles)
    return tile, max(1, min(splits, M // 512))


class Conv3x3(torch.autograd.Function):
    """Stride-1 3x3 convolution (pad 1) on the hand-written implicit-GEMM
    kernels (csrc/kernels/conv_igemm.hip streaming kernel: any H, W), reading
    the channels-last shadow ``bind.wcl`` ([Cout][3][3][Cin] in memory) and a
    zero-bordered input; the weight gradient is split-K slabs reduce-added into
    the flat gradient in PyTorch's [Cout][Cin][3][3] order.  The padded input
    and the padded output gradient come straight from the BatchNorm kernels
    (bn_act out_pad / dx_pad) when the model wires them, else from a pad copy.
    ``stats``: fp32 [2*Cout] <- the output's per-channel sum / sum of squares
    (GEMM epilogue rows, as Conv1x1)."""

    @staticmethod
    def forward(ctx, x, weight, bind: ShadowBinding, stats):
        C = native()
        N, cin, H, W = x.shape
        cout = weight.shape[0]
        keep, xbase = _padded_base(x, 1)
        M, K = N * H * W, 9 * cin
        y = torch.empty((N, cout, H, W), dtype=BF16, device=x.device, memory_format=torch.channels_last)
        tile, splits = _plan_3x3(M, cout, K)
        slab = torch.empty(splits * M * cout, device=x.device) if splits > 1 else None
        rows = None
        s = stream_handle()
        if stats is not None:
            if C.reduce_atomic() != 0:
                raise RuntimeError("Conv3x3 statistics need reduction mode 0 (partial rows)")
            nrows = C.conv_fwd_stat_rows(N, H, W, cin, cout, 3, tile, splits)
            rows = torch.empty(max(nrows, 400 if splits > 1 else 1), 2, cout, device=x.device)
        T = C.conv_fwd(xbase, bind.wcl.data_ptr(), y.data_ptr(), 0 if rows is None else rows.data_ptr(),
                       0 if slab is None else slab.data_ptr(), N, H, W, cin, cout, 3, tile, splits, s)
        if rows is not None:
            C.bn_rows_reduce(rows.data_ptr(), T, cout, stats.data_ptr(), s)
        ctx.save_for_backward(keep)
        ctx.xbase, ctx.bind, ctx.geom = xbase, bind, (N, cin, H, W, cout)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        N, cin, H, W, cout = ctx.geom
        bind = ctx.bind
        s = stream_handle()
        keep_dy, dybase = _padded_base(dy, 1)
        M, K = N * H * W, 9 * cin
        dx = None
        if ctx.needs_input_grad[0]:
            wt = torch.empty(cin, 3, 3, cout, dtype=BF16, device=dy.device)
            C.weight_flip_transpose(bind.wcl.data_ptr(), wt.data_ptr(), cout, cin, 3, s)
            dx = torch.empty((N, cin, H, W), dtype=BF16, device=dy.device, memory_format=torch.channels_last)
            dt, ds = _plan_3x3(M, cin, 9 * cout)
            slab = torch.empty(ds * M * cin, device=dy.device) if ds > 1 else None
            C.conv_fwd(dybase, wt.data_ptr(), dx.data_ptr(), 0, 0 if slab is None else slab.data_ptr(), N, H, W,
                       cout, cin, 3, dt, ds, s)
        tile, splits = _wgrad_plan_3x3(cout, K, M)
        ws = torch.empty(splits * cout * K, device=dy.device)
        C.conv_wgrad(dybase, ctx.xbase, ws.data_ptr(), N, H, W, cin, cout, 3, splits, K, tile, 0, s)
        C.slab_reduce_add_oihw(ws.data_ptr(), bind.g32.data_ptr(), splits, cout, 9, cin, cin, s)
        bind.ready()
        del keep_dy
        return dx, None, None, None


class ShadowConv(torch.autograd.Function):
    """MIOpen convolution on the bf16 shadow weight; fp32 weight gradient
    added into the flat buffer."""

    @staticmethod
    def forward(ctx, x, weight, bind: ShadowBinding, stride: int, pad: int, dx_sink=None):
        w16 = bind.wcl if bind.wcl is not None else bind.w16.view(weight.shape)
        ctx.dx_sink = dx_sink
        if dx_sink is not None:
            dx_sink["expect"] = True
        ctx.save_for_backward(x)
        ctx.bind, ctx.stride, ctx.pad, ctx.wshape = bind, stride, pad, weight.shape
        return F.conv2d(x, w16, None, stride, pad)

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        bind = ctx.bind
        w16 = bind.wcl if bind.wcl is not None else bind.w16.view(ctx.wshape)
        dx, dw, _ = torch.ops.aten.convolution_backward(
            dy, x, w16, None, (ctx.stride, ctx.stride), (ctx.pad, ctx.pad), (1, 1), False, (0, 0), 1,
            (ctx.needs_input_grad[0], True, False))
        bind.g32.view(ctx.wshape).add_(dw)
        bind.ready()
        if ctx.dx_sink is not None and dx is not None and not ctx.dx_sink.get("done"):
            # the same input feeds a 1x1 conv whose dgrad epilogue adds this (ResNet
            # downsample blocks: no separate sum of the two input gradients)
            ctx.dx_sink["g"] = dx
            dx = None
        return dx, None, None, None, None, None


# ---------------------------------------------------------------------------
# strided convolutions and the stem on the generalised MFMA kernels
# (csrc conv_fwd_ex / conv_wgrad_ex): no MIOpen convolution in the ResNet-50
# training step
# ---------------------------------------------------------------------------
def _stream():
    return stream_handle()


class StemConv(torch.autograd.Function):
    """The ResNet-50 stem: 7x7 stride-2 pad-3 conv over 3 input channels.
    A stride-2 conv over a 2x2 space-to-depth image is a stride-1 conv: the
    padded image becomes S[n][i][j][(a*2+b)*3 + c] = x[n][2i+a-3][2j+b-3][c]
    (12 channels, zero-padded to 16: one 32-byte vector per pixel) and the
    7x7 weights a 4x4x16 kernel (zero taps past 7), so the stem runs as a
    4x4 stride-1 implicit GEMM with K = 256 on the MFMA kernels (csrc
    resnet_glue.hip s2d_stem_input / stem_weight_pack / stem_wgrad_unpack).
    No input gradient (the image).  ``stats``: BN sum / sum of squares rows."""

    @staticmethod
    def forward(ctx, x, weight, bind: ShadowBinding, stats):
        C = native()
        N, cin, H, W = x.shape
        if cin != 3 or not x.is_contiguous(memory_format=torch.channels_last) or x.dtype != BF16:
            raise ValueError("StemConv: channels-last bf16 [N, 3, H, W] input")
        cout = weight.shape[0]
        Ho, Wo = (H + 6 - 7) // 2 + 1, (W + 6 - 7) // 2 + 1
        Hs, Ws = Ho + 3, Wo + 3
        s = _stream()
        S = torch.empty(N, Hs, Ws, 16, dtype=BF16, device=x.device)
        C.s2d_stem_input(x.data_ptr(), S.data_ptr(), N, H, W, Hs, Ws, 3, s)
        w4 = torch.empty(cout, 4, 4, 16, dtype=BF16, device=x.device)
        C.stem_weight_pack(bind.w16.data_ptr(), w4.data_ptr(), cout, s)
        y = torch.empty((N, cout, Ho, Wo), dtype=BF16, device=x.device, memory_format=torch.channels_last)
        tile = 0 if cout % 128 == 0 else 2
        rows = None
        if stats is not None:
            if C.reduce_atomic() != 0:
                raise RuntimeError("StemConv statistics need reduction mode 0 (partial rows)")
            rows = torch.empty((N * Ho * Wo + 127) // 128, 2, cout, device=x.device)
        T = C.conv_fwd_ex(S.data_ptr(), w4.data_ptr(), y.data_ptr(), 0 if rows is None else rows.data_ptr(), 0, N, Ho,
                          Wo, Hs, Ws, 16, cout, 4, 4, 1, 0, 0, 0, 0, 0, 0, tile, 1, s)
        if rows is not None:
            C.bn_rows_reduce(rows.data_ptr(), T, cout, stats.data_ptr(), s)
        ctx.save_for_backward(S)
        ctx.bind, ctx.geom = bind, (N, Ho, Wo, Hs, Ws, cout)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        (S,) = ctx.saved_tensors
        N, Ho, Wo, Hs, Ws, cout = ctx.geom
        s = _stream()
        dy = dy.contiguous(memory_format=torch.channels_last)
        tile, splits = _wgrad_plan_3x3(cout, 256, N * Ho * Wo)
        ws = torch.empty(splits * cout * 256, device=dy.device)
        C.conv_wgrad_ex(dy.data_ptr(), S.data_ptr(), ws.data_ptr(), N, Ho, Wo, Hs, Ws, Ho, Wo, 0, 16, cout, 4, 4, 1,
                        splits, 256, tile, s)
        C.stem_wgrad_unpack(ws.data_ptr(), ctx.bind.g32.data_ptr(), splits, cout, s)
        ctx.bind.ready()
        return None, None, None, None


class Conv1x1S2(torch.autograd.Function):
    """Stride-2 1x1 convolution (the ResNet-50 downsample) as an implicit GEMM
    whose rows read every other pixel of the unpadded input (conv_fwd_ex,
    S = 2): no gather copy.  Weight gradient: conv_wgrad_ex (stride-2 rows).
    Input gradient: nonzero only at the even pixels, dx[2q] = dy[q] W --
    handed to the c1 (stride-1 1x1) conv of the same block, whose backward
    accumulates it IN PLACE into its own dx at those rows (the GEMM
    epilogue's output map + addend = dx itself: no zero-filled full-size
    tensor, no elementwise sum).  If c1's backward already ran (autograd
    gives no ordering guarantee), the gradient is materialised and returned
    through autograd instead."""

    @staticmethod
    def forward(ctx, x, weight, bind: ShadowBinding, stats, dx_sink=None):
        C = native()
        x = x.contiguous(memory_format=torch.channels_last)
        N, cin, H, W = x.shape
        cout = weight.shape[0]
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        ctx.dx_sink = dx_sink
        if dx_sink is not None:
            dx_sink["expect"] = True
        y = torch.empty((N, cout, Ho, Wo), dtype=BF16, device=x.device, memory_format=torch.channels_last)
        tile = 0 if cout % 128 == 0 else 2
        s = _stream()
        rows = None
        if stats is not None:
            if C.reduce_atomic() != 0:
                raise RuntimeError("Conv1x1S2 statistics need reduction mode 0 (partial rows)")
            rows = torch.empty((N * Ho * Wo + 127) // 128, 2, cout, device=x.device)
        T = C.conv_fwd_ex(x.data_ptr(), bind.w16.data_ptr(), y.data_ptr(), 0 if rows is None else rows.data_ptr(), 0,
                          N, Ho, Wo, H, W, cin, cout, 1, 1, 2, 0, 0, 0, 0, 0, 0, tile, 1, s)
        if rows is not None:
            C.bn_rows_reduce(rows.data_ptr(), T, cout, stats.data_ptr(), s)
        ctx.save_for_backward(x)
        ctx.bind, ctx.geom = bind, (N, cin, H, W, cout, Ho, Wo)
        return y

    @staticmethod
    def deferred_dgrad(C, dy, wt, geom, dx, s):
        """dx[:, 0::2, 0::2] += dy W (in place, bf16) -- the c1 conv's backward calls this."""
        N, cin, H, W, cout, Ho, Wo = geom
        tile = 0 if cin % 128 == 0 else 2
        C.conv_fwd_ex(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, 0, N, Ho, Wo, Ho, Wo, cout, cin, 1, 1, 1, 2, 0, 0,
                      W, H * W, dx.data_ptr(), tile, 1, s)

    @staticmethod
    def backward(ctx, dy):
        C = native()
        (x,) = ctx.saved_tensors
        bind = ctx.bind
        N, cin, H, W, cout, Ho, Wo = ctx.geom
        s = _stream()
        dy = dy.contiguous(memory_format=torch.channels_last)
        M = N * Ho * Wo
        tile, splits = _wgrad_plan(cout, cin, M)
        ws = torch.empty(splits * cout * cin, device=x.device)
        C.conv_wgrad_ex(dy.data_ptr(), x.data_ptr(), ws.data_ptr(), N, Ho, Wo, H, W, Ho, Wo, 0, cin, cout, 1, 1, 2,
                        splits, cin, tile, s)
        C.slab_reduce_add(ws.data_ptr(), bind.g32.data_ptr(), splits, cout, 1, cin, cin, s)
        bind.ready()
        if not ctx.needs_input_grad[0]:
            return None, None, None, None, None
        wt = bind.wt
        if wt is None:
            wt = torch.empty(cin, cout, dtype=BF16, device=x.device)
            C.weight_flip_transpose(bind.w16.data_ptr(), wt.data_ptr(), cout, cin, 1, s)
        sink = ctx.dx_sink
        if sink is not None and not sink.get("done"):
            sink["s2"] = (dy, wt, ctx.geom)  # accumulated by the c1 dgrad (Conv1x1.backward)
            return None, None, None, None, None
        dx = torch.zeros_like(x, memory_format=torch.channels_last)
        Conv1x1S2.deferred_dgrad(C, dy, wt, ctx.geom, dx, s)
        return dx, None, None, None, None


class Conv3x3S2(torch.autograd.Function):
    """Stride-2 3x3 pad-1 convolution (the first bottleneck of stages 2-4)
    on the generalised MFMA kernels: forward and weight gradient read the
    zero-bordered input with stride-2 rows (conv_fwd_ex / conv_wgrad_ex).
    Input gradient by output parity: dx[2q + r] (per axis) only sees the
    kernel taps of parity r -- 1 tap for r = 0, 2 for r = 1 -- so it is four
    phase convolutions (1x1, 1x2, 2x1, 2x2 over the zero-bordered dy, weights
    from csrc phase_weights) each storing its pixels interleaved into dx
    through the epilogue's output map: exactly the 9 taps of work, no
    zero-stuffed upsampling."""

    @staticmethod
    def forward(ctx, x, weight, bind: ShadowBinding, stats):
        C = native()
        N, cin, H, W = x.shape
        cout = weight.shape[0]
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        keep, xbase = _padded_base(x, 1)
        y = torch.empty((N, cout, Ho, Wo), dtype=BF16, device=x.device, memory_format=torch.channels_last)
        tile = 0 if cout % 128 == 0 else 2
        s = _stream()
        rows = None
        if stats is not None:
            if C.reduce_atomic() != 0:
                raise RuntimeError("Conv3x3S2 statistics need reduction mode 0 (partial rows)")
            rows = torch.empty((N * Ho * Wo + 127) // 128, 2, cout, device=x.device)
        T = C.conv_fwd_ex(xbase, bind.wcl.data_ptr(), y.data_ptr(), 0 if rows is None else rows.data_ptr(), 0, N, Ho,
                          Wo, H + 2, W + 2, cin, cout, 3, 3, 2, 0, 0, 0, 0, 0, 0, tile, 1, s)
        if rows is not None:
            C.bn_rows_reduce(rows.data_ptr(), T, cout, stats.data_ptr(), s)
        ctx.save_for_backward(keep)
        ctx.xbase, ctx.bind, ctx.geom = xbase, bind, (N, cin, H, W, cout, Ho, Wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        C = native()
        N, cin, H, W, cout, Ho, Wo = ctx.geom
        bind = ctx.bind
        s = _stream()
        keep_dy, dybase = _padded_base(dy, 1)  # [N][Ho+2][Wo+2][cout], interior at (1, 1)
        Hq, Wq = Ho + 2, Wo + 2
        dx = None
        if ctx.needs_input_grad[0]:
            if H != 2 * Ho or W != 2 * Wo:
                raise ValueError("Conv3x3S2: even input sizes only")
            wt = torch.empty(cin, 3, 3, cout, dtype=BF16, device=dy.device)
            C.weight_flip_transpose(bind.wcl.data_ptr(), wt.data_ptr(), cout, cin, 3, s)
            ph = torch.empty(9 * cin * cout, dtype=BF16, device=dy.device)
            C.phase_weights(wt.data_ptr(), ph.data_ptr(), cin, cout, s)
            dx = torch.empty((N, cin, H, W), dtype=BF16, device=dy.device, memory_format=torch.channels_last)
            interior = dybase + (Wq + 1) * cout * 2  # dy[0][0]: tap t of phase pixel q reads dy[q + t]
            tile = 0 if cin % 128 == 0 else 2
            off = 0
            for rh in (0, 1):
                for rw in (0, 1):
                    kh, kw = 1 + rh, 1 + rw
                    C.conv_fwd_ex(interior, ph[off * cin * cout:].data_ptr(), dx.data_ptr(), 0, 0, N, Ho, Wo, Hq, Wq,
                                  cout, cin, kh, kw, 1, 2, rh, rw, W, H * W, 0, tile, 1, s)
                    off += kh * kw
        K = 9 * cin
        tile_w, splits = _wgrad_plan_3x3(cout, K, N * Ho * Wo)
        ws = torch.empty(splits * cout * K, device=dy.device)
        C.conv_wgrad_ex(dybase, ctx.xbase, ws.data_ptr(), N, Ho, Wo, H + 2, W + 2, Hq, Wq, 1, cin, cout, 3, 3, 2,
                        splits, K, tile_w, s)
        C.slab_reduce_add_oihw(ws.data_ptr(), bind.g32.data_ptr(), splits, cout, 9, cin, cin, s)
        bind.ready()
        del keep_dy
        return dx, None, None, None
