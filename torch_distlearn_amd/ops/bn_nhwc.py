"""Fused channels-last training BatchNorm (+ReLU, +residual add) on the HIP
kernels of ``csrc/kernels/bn_nhwc.hip`` -- the ResNet-50 path's BN.

``bn_act(x, weight, bias, running_mean, running_var, residual=None, relu=True)``
computes ``act(BN(x) [+ residual])`` for a channels-last bf16 ``x`` [N, C, H, W]
with fp32 statistics / affine parameters, updating the running statistics like
``F.batch_norm(training=True)``.  Backward fuses the ReLU mask, the BN input
gradient and the residual gradient into two kernels.  Reference parity: the
reference's cunn ``SpatialBatchNormalization`` + ``ReLU`` layers
(examples/cifar10.lua:108-133); numerics are tested against the fp32 PyTorch
op (tests/kernels/test_resnet_gpu.py).
"""
from __future__ import annotations

import weakref
from typing import Optional

import torch

from .._native import native, stream_handle

# BN + residual + ReLU keeps its ReLU mask as bits for the backward (relu mode 3)
# instead of re-reading the output y in both backward passes; False = mode 1 (A/B)
_MASK_BITS = True
# ... and hands (dy, mask bits) to the residual's consumer instead of writing
# the residual gradient (False: writes dres -- the tests' reference path)
_MASKED_ADDEND = True


def unpack_mask_bits(mbits: torch.Tensor, shape_like: torch.Tensor) -> torch.Tensor:
    """bool [N, C, H, W] (channels-last) from relu mode 3's mask bits
    (uint8 [M][C/8], bit k of byte (m, j) = channel 8j + k)."""
    n, c, h, w = shape_like.shape
    sh = torch.arange(8, device=mbits.device, dtype=torch.uint8)
    bits = ((mbits.view(-1, c // 8, 1) >> sh) & 1).view(n, h, w, c).bool()
    return bits.permute(0, 3, 1, 2)


def _bn():
    return native()


def _geom(x: torch.Tensor):
    n, c, h, w = x.shape
    return n * h * w, c


def padded_empty(n: int, c: int, h: int, w: int, pad: int, device) -> torch.Tensor:
    """A [N, C, H, W] channels-last bf16 view of the interior of a fresh
    [N, H+2p, W+2p, C] buffer whose border ring is zeroed: the zero-bordered
    layout the implicit-GEMM 3x3 kernels read directly (ops/conv.py Conv3x3).
    The view carries ``_dl_pad = pad`` so consumers can find the buffer."""
    hp, wp = h + 2 * pad, w + 2 * pad
    buf = torch.empty((n, hp, wp, c), dtype=torch.bfloat16, device=device)
    native().zero_border_nhwc(buf.data_ptr(), n, h, w, c, pad, stream_handle())
    v = buf.as_strided((n, c, h, w), (hp * wp * c, 1, wp * c, c), (pad * wp + pad) * c)
    v._dl_pad = pad
    return v


def padded_buffer(cache: dict, role: str, n: int, c: int, h: int, w: int, pad: int, device) -> torch.Tensor:
    """:func:`padded_empty` whose buffer persists in ``cache`` (a dict the
    owner keeps, e.g. the BatchNorm module's) per (role, shape): its border is
    zeroed once instead of by a zero_border launch per use (32 per ResNet-50
    step).  Each call returns a fresh view of the cached buffer -- unless the
    previous view is still alive (weakref), e.g. saved by a backward that has
    not run yet, in which case the call gets a fresh buffer of its own."""
    k = (role, n, c, h, w, pad, str(device))
    ent = cache.get(k)
    if ent is not None and ent[1]() is not None:
        # the previous view is still referenced (e.g. saved for a backward that
        # has not run: two forwards before one backward): a fresh buffer this time
        return padded_empty(n, c, h, w, pad, device)
    if ent is None:
        ent = [padded_empty(n, c, h, w, pad, device), lambda: None]
        cache[k] = ent
    base = ent[0]
    hp, wp = h + 2 * pad, w + 2 * pad
    v = base.as_strided((n, c, h, w), (hp * wp * c, 1, wp * c, c), base.storage_offset())
    v._dl_pad = pad
    ent[1] = weakref.ref(v)
    return v


def supported(x: torch.Tensor) -> bool:
    c = x.shape[1]
    ok_c = c % 8 == 0 and ((c < 256 and 256 % (c // 8) == 0) or c % 256 == 0)
    return (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and ok_c
            and x.is_contiguous(memory_format=torch.channels_last))


def materialize(t: torch.Tensor) -> torch.Tensor:
    """Run the deferred apply of a BatchNorm output made with ``defer_apply``
    or ``defer_pool`` (for a consumer that cannot apply it on load); returns ``t``."""
    for key in ("_dl_res_bn", "_dl_pool_bn"):
        args = getattr(t, key, None)
        if args is not None:
            delattr(t, key)
            _bn().bn_nhwc_fwd_pad(*args[0], stream_handle(), 0)
    return t


class _BnAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, residual, relu, eps, momentum, acc, grads, res_sink,
                have_stats, out_pad, dx_pad, bn_link, on_load=False, defer_apply=False, defer_pool=False,
                pad_key=None):
        M, C = _geom(x)
        N, _, H, W = x.shape
        ctx.pad_key = pad_key
        if out_pad:
            y = (padded_buffer(pad_key, "y", N, C, H, W, out_pad, x.device) if pad_key is not None
                 else padded_empty(N, C, H, W, out_pad, x.device))
        else:
            y = torch.empty_like(x, memory_format=torch.channels_last)
        ctx.dx_pad = dx_pad
        # forward and backward per-channel sums in one zeroed buffer (one fill, or a
        # slice of the caller's per-step zeroed arena); with have_stats the first 2C
        # already hold the forward statistics (emitted by the producing convolution's
        # epilogue): the statistics pass is skipped
        if acc is None:
            acc = torch.zeros(4 * C, device=x.device, dtype=torch.float32)
            have_stats = False
        ctx.backwards = 0
        save = torch.empty(2 * C, device=x.device, dtype=torch.float32)
        # a residual that is a deferred BatchNorm output (the downsample branch's BN,
        # defer_apply): this apply reads that BN's input and applies it on load
        rbn = getattr(residual, "_dl_res_bn", None) if residual is not None else None
        if rbn is not None:
            del residual._dl_res_bn
            res = rbn[1][0]
        else:
            res = residual.contiguous(memory_format=torch.channels_last) if residual is not None else None
        # (with out_pad the kernel writes y's padded buffer: its origin is y.data_ptr()
        # minus the interior offset)
        ybase = y.data_ptr() - (out_pad * (W + 2 * out_pad) + out_pad) * C * 2 if out_pad else y.data_ptr()
        # BN + residual + ReLU: the backward needs the output's ReLU mask, which x
        # alone does not give.  The apply writes it as bits (one byte per 8
        # channels per row, 1/16 of y) so both backward passes read that instead
        # of y (relu mode 3); y itself is then not kept for the backward (a
        # consuming c1 dgrad adds the residual gradient under the bits too).
        mbits = None
        if relu and residual is not None and _MASK_BITS:
            mbits = torch.empty(M * C // 8, dtype=torch.uint8, device=x.device)
        apply = (x.data_ptr(), res.data_ptr() if res is not None else 0, ybase, acc.data_ptr(),
                 weight.data_ptr(), bias.data_ptr(), save.data_ptr(),
                 running_mean.data_ptr() if running_mean is not None else 0,
                 running_var.data_ptr() if running_var is not None else 0, M, C, float(eps), float(momentum),
                 int(relu), int(have_stats), H, W, int(out_pad))
        if defer_pool and relu and residual is None and have_stats and not out_pad and mbits is None:
            # y feeds the stem max-pool, which applies this BN + ReLU on load (csrc
            # pool_nhwc.hip PoolBn); the backward needs neither y nor its mask (relu 2)
            y._dl_pool_bn = (apply, (x, acc, weight, bias, save, running_mean, running_var, eps, momentum))
        elif defer_apply and not relu and residual is None and have_stats and not out_pad:
            # y is the residual of a BN + residual + ReLU whose apply applies this BN
            # on load (its kernel publishes save and the running statistics); y stays
            # unwritten unless a consumer calls materialize()
            y._dl_res_bn = (apply, (x, acc, weight, bias, save, running_mean, running_var, eps, momentum))
        else:
            rargs = {}
            if rbn is not None:
                _, racc, rw, rb, rsave, rrm, rrv, reps, rmom = rbn[1]
                rargs = dict(rbn_acc=racc.data_ptr(), rbn_w=rw.data_ptr(), rbn_b=rb.data_ptr(),
                             rbn_save=rsave.data_ptr(), rbn_rm=rrm.data_ptr() if rrm is not None else 0,
                             rbn_rv=rrv.data_ptr() if rrv is not None else 0, rbn_eps=float(reps),
                             rbn_momentum=float(rmom))
            _bn().bn_nhwc_fwd_pad(*apply, stream_handle(), mbits.data_ptr() if mbits is not None else 0, **rargs)
        ctx.has_res = residual is not None
        # the residual branch's BN backward fused into this backward (csrc ResBnBwd):
        # a BN + residual + ReLU takes it over from a defer_apply BN that made its residual
        ctx.rbn_bwd = None
        if residual is not None and getattr(residual, "_dl_res_bwd", None) is not None:
            ctx.rbn_bwd = residual._dl_res_bwd
            del residual._dl_res_bwd
        ctx.own_link = None
        if defer_apply and not relu and residual is None and not out_pad:
            ctx.own_link = {"fwd": (x, save, weight, bias, acc, grads)}
            y._dl_res_bwd = ctx.own_link
        elif getattr(y, "_dl_pool_bn", None) is not None:
            # ... and the stem max-pool's backward computes this BN's backward too
            # (csrc pool_nhwc.hip maxpool3s2_bwd_bn_kernel; relu mode 2)
            ctx.own_link = {"fwd": (x, save, weight, bias, acc, grads)}
            y._dl_pool_bwd = ctx.own_link
        ctx.grads = grads
        ctx.res_sink = res_sink
        if res_sink is not None and residual is not None:
            res_sink["expect"] = True  # the residual's gradient goes to the sink, not to autograd
        # relu mask: from the output when a residual was added (mode 1),
        # otherwise recomputed from x in the backward kernels (mode 2: y is
        # neither saved nor read)
        ctx.relu = (3 if mbits is not None else 1 if ctx.has_res else 2) if relu else 0
        ctx.save_for_backward(x, y if ctx.relu == 1 else mbits, weight, bias, save, acc)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, weight, bias, save, acc4 = ctx.saved_tensors
        M, C = _geom(x)
        if ctx.own_link is not None and ctx.own_link.pop("fused", None):
            # the consuming BN + residual + ReLU's backward already computed this BN's
            # input gradient (it arrives as dy) and its dgamma / dbeta
            dw, db = ctx.own_link.pop("dwdb")
            if ctx.grads is not None:
                ctx.grads[2]()
                return (dy, None, None, None, None, None, None, None, None, None, None, None, None, None, None, None,
                        None, None, None, None)
            return (dy, dw.to(weight.dtype), db.to(weight.dtype), None, None, None, None, None, None, None, None, None,
                    None, None, None, None, None, None, None, None)
        dy = dy.contiguous(memory_format=torch.channels_last)
        N, _, H, W = x.shape
        p = ctx.dx_pad
        if p:
            dx = (padded_buffer(ctx.pad_key, "dx", N, C, H, W, p, x.device) if ctx.pad_key is not None
                  else padded_empty(N, C, H, W, p, x.device))
        else:
            dx = torch.empty_like(x, memory_format=torch.channels_last)
        dxbase = dx.data_ptr() - (p * (W + 2 * p) + p) * C * 2 if p else dx.data_ptr()
        # relu mode 3 with a waiting consumer (the conv whose input is the residual,
        # ops/conv.py Conv1x1): the residual gradient dy * mask is not written
        # here -- the consumer's dgrad epilogue adds dy under the mask bits itself
        # (one full write + read of dres fewer)
        park = (ctx.relu == 3 and ctx.res_sink is not None and _MASKED_ADDEND and ctx.has_res
                and not ctx.res_sink.get("done"))
        dres = torch.empty_like(x, memory_format=torch.channels_last) if (ctx.has_res and not park) else None
        acc = acc4[2 * C:]
        have_sums = False  # (the dgrad-epilogue sums of round 5 were removed in round 6)
        if ctx.backwards and not have_sums:  # the kernels accumulate atomically into the zeroed
            acc.zero_()                       # half: a second backward (retain_graph) restarts at 0
        ctx.backwards += 1
        if ctx.grads is not None:  # dgamma / dbeta straight into the flat gradient (overwritten)
            dw, db, ready = ctx.grads
        else:
            dw = torch.empty(C, device=x.device, dtype=torch.float32)
            db = torch.empty(C, device=x.device, dtype=torch.float32)
        ym = y if ctx.relu == 1 else None      # (the saved slot holds the mask bits in relu mode 3)
        mb = y if ctx.relu == 3 else None
        rargs = {}
        rl = ctx.rbn_bwd
        if rl is not None and dres is not None and not have_sums and "fwd" in rl:
            # dres <- the residual BN's input gradient (its reduce sums ride our reduce pass)
            rx, rsave, rw, _, racc4, rgrads = rl["fwd"]
            rC = rx.shape[1]
            racc = racc4[2 * rC:]
            if ctx.backwards > 1:
                racc.zero_()
            if rgrads is not None:
                rdw, rdb = rgrads[0], rgrads[1]
            else:
                rdw = torch.empty(rC, device=x.device, dtype=torch.float32)
                rdb = torch.empty(rC, device=x.device, dtype=torch.float32)
            rargs = dict(rbn_x=rx.data_ptr(), rbn_save=rsave.data_ptr(), rbn_w=rw.data_ptr(), rbn_acc=racc.data_ptr(),
                         rbn_dw=rdw.data_ptr(), rbn_db=rdb.data_ptr())
            rl["fused"] = True
            rl["dwdb"] = (rdw, rdb)
        _bn().bn_nhwc_bwd_pad(dy.data_ptr(), ym.data_ptr() if ym is not None else 0, x.data_ptr(), save.data_ptr(),
                                 weight.data_ptr(), bias.data_ptr(), acc.data_ptr(), dxbase,
                                 dres.data_ptr() if dres is not None else 0, dw.data_ptr(), db.data_ptr(), M, C,
                                 ctx.relu, H, W, int(p), stream_handle(), int(have_sums),
                                 mb.data_ptr() if mb is not None else 0, **rargs)
        if park:
            ctx.res_sink["gm"] = (dy, mb)
        elif ctx.res_sink is not None and dres is not None and not ctx.res_sink.get("done"):
            # consumed by the conv whose input is the residual (ops/conv.py); if that
            # conv's backward already ran ("done"), autograd sums the gradients instead
            ctx.res_sink["g"] = dres
            dres = None
        if ctx.grads is not None:
            ready()
            return (dx, None, None, None, None, dres, None, None, None, None, None, None, None, None, None, None, None,
                    None, None, None)
        return (dx, dw.to(weight.dtype), db.to(weight.dtype), None, None, dres, None, None, None, None, None, None, None,
                None, None, None, None, None, None, None)


@torch.no_grad()
def bn_act_eval(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, running_mean: torch.Tensor,
                running_var: torch.Tensor, residual: Optional[torch.Tensor] = None, relu: bool = True,
                eps: float = 1e-5, out_pad: int = 0) -> torch.Tensor:
    """Eval-mode ``act(BN(x) [+ residual])`` from the running statistics on
    the same HIP apply kernel as training (the ResNet-50 predict path; no
    fp32 copy, no MIOpen): the kernel derives mean / variance from a [2C]
    (sum, sum of squares) pair, so it is given M*mean and M*(var + mean^2)
    of the running statistics and the statistics pass is skipped.  No
    running-statistics update; not differentiable."""
    M, C = _geom(x)
    N, _, H, W = x.shape
    rm, rv = running_mean.float(), running_var.float()
    acc = torch.cat([rm * M, (rv + rm * rm) * M])
    save = torch.empty(2 * C, device=x.device, dtype=torch.float32)
    y = padded_empty(N, C, H, W, out_pad, x.device) if out_pad else torch.empty_like(x, memory_format=torch.channels_last)
    ybase = y.data_ptr() - (out_pad * (W + 2 * out_pad) + out_pad) * C * 2 if out_pad else y.data_ptr()
    res = residual.contiguous(memory_format=torch.channels_last) if residual is not None else None
    _bn().bn_nhwc_fwd_pad(x.data_ptr(), res.data_ptr() if res is not None else 0, ybase, acc.data_ptr(),
                          weight.contiguous().data_ptr(), bias.contiguous().data_ptr(), save.data_ptr(), 0, 0, M, C,
                          float(eps), 0.0, int(relu), 1, H, W, int(out_pad), stream_handle())
    return y


def bn_act(x: torch.Tensor, weight: torch.Tensor, bias: torch.Tensor, running_mean: Optional[torch.Tensor],
           running_var: Optional[torch.Tensor], residual: Optional[torch.Tensor] = None, relu: bool = True,
           eps: float = 1e-5, momentum: float = 0.1, acc: Optional[torch.Tensor] = None,
           grads=None, res_sink: Optional[dict] = None, have_stats: Optional[bool] = None, out_pad: int = 0,
           dx_pad: int = 0, defer_apply: bool = False, defer_pool: bool = False, pad_key=None) -> torch.Tensor:
    """``acc``: optional fp32 [4C] whose last 2C are zero; with ``have_stats``
    (the default when ``acc`` is given) its first 2C already hold the
    per-channel sum / sum of squares of x (see ops/conv.py Conv1x1), else they
    are zero too and the statistics pass fills them.
    ``grads``: optional (dweight view, dbias view, ready callback): the
    backward writes the parameter gradients there (e.g. into the flat
    gradient buffer) instead of returning them to autograd.
    ``res_sink``: a dict that receives the residual's gradient (key ``"g"``)
    instead of autograd, for a consumer that adds it itself (Conv1x1's dgrad
    epilogue): saves the separate gradient-sum pass of a tensor used twice.
    ``out_pad`` / ``dx_pad``: write the output / the input gradient as the
    interior of a zero-bordered buffer (:func:`padded_empty`) for a 3x3
    convolution that reads it directly.
    ``defer_apply`` (no ReLU, no residual, statistics given, unpadded): the
    returned tensor is only a handle for the BN + residual + ReLU that takes it
    as its residual -- that apply reads this BN's input and applies it on load
    (csrc ResBn), so this apply launch and the write + read of its output go;
    :func:`materialize` runs it for any other consumer.
    ``defer_pool`` (ReLU, no residual, statistics given, unpadded): the same
    for the stem max-pool (ops/pool.py), which applies this BN + ReLU to the
    window elements it loads (csrc pool_nhwc.hip PoolBn).
    ``pad_key``: a dict in which the zero-bordered output / input gradient
    buffers persist (:func:`padded_buffer`; the BatchNorm module's): no border
    fill per use."""
    if not supported(x):
        raise ValueError(f"bn_act: needs a channels-last bf16 CUDA tensor with a supported channel count, got "
                         f"{tuple(x.shape)} {x.dtype} {x.device}")
    if residual is not None and (residual.shape != x.shape or residual.dtype != x.dtype):
        raise ValueError("bn_act: residual must match x in shape and dtype")
    if residual is not None and getattr(residual, "_dl_res_bn", None) is not None and out_pad:
        materialize(residual)
    if weight.dtype != torch.float32 or bias.dtype != torch.float32:
        raise ValueError("bn_act: weight / bias must be fp32")
    if acc is not None and (acc.numel() != 4 * x.shape[1] or acc.dtype != torch.float32):
        raise ValueError("bn_act: acc must be fp32 [4C]")
    if out_pad and residual is not None:
        raise ValueError("bn_act: out_pad with a residual is not supported (the backward reads y linearly)")
    if have_stats is None:
        have_stats = acc is not None
    return _BnAct.apply(x, weight.contiguous(), bias.contiguous(), running_mean, running_var, residual, relu, eps,
                        momentum, acc, grads, res_sink, bool(have_stats), int(out_pad), int(dx_pad),
                        None, False, bool(defer_apply), bool(defer_pool), pad_key)
