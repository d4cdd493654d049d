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
        native().maxpool_nhwc_fwd(x.data_ptr(), y.data_ptr(), idx.data_ptr(), N, H, W, C, k, s, p, stream_handle())
        ctx.save_for_backward(idx)
        ctx.geom = (N, C, H, W, k, s, p)
        return y

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        N, C, H, W, k, s, p = ctx.geom
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = torch.empty((N, C, H, W), dtype=dy.dtype, device=dy.device, memory_format=torch.channels_last)
        native().maxpool_nhwc_bwd(dy.data_ptr(), idx.data_ptr(), dx.data_ptr(), N, H, W, C, k, s, p, stream_handle())
        return dx, None, None, None


def max_pool2d_nhwc(x: torch.Tensor, k: int, s: int, p: int) -> torch.Tensor:
    if not supported(x):
        raise ValueError("max_pool2d_nhwc: needs a channels-last bf16 CUDA tensor with C % 8 == 0")
    return _MaxPool.apply(x, k, s, p)
