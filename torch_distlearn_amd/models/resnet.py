"""ResNet-50 (ImageNet shape, 25.6M parameters) -- BASELINE.json config 5:
"ResNet-50 ImageNet-shape synthetic AllReduceSGD bf16 (bucket fusion / xGMI
bandwidth stress)".  Not a model of the reference; it exists to exercise the
bucketed gradient all-reduce with a 102 MB fp32 gradient (~25 MB
buckets, >= 4 per step).

Compute path: PyTorch ops (MIOpen) in channels-last bf16 with fp32 master
weights in the flat buffer; BatchNorm in fp32 statistics.  Parameters are
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


class _BN(nn.Module):
    def __init__(self, c: int, zero: bool = False):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(c) if zero else torch.ones(c))
        self.bias = nn.Parameter(torch.zeros(c))
        self.register_buffer("running_mean", torch.zeros(c))
        self.register_buffer("running_var", torch.ones(c))

    def forward(self, x):
        if _BN_MODE == "mixed" and x.is_cuda:
            return F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias, self.training, 0.1,
                                1e-5)
        y = F.batch_norm(x.float(), self.running_mean, self.running_var, self.weight, self.bias, self.training, 0.1,
                         1e-5)
        return y.to(x.dtype)

    def act(self, x, relu: bool = True, residual=None):
        """act(BN(x) [+ residual]); one fused HIP kernel pair in "hip" mode."""
        if _BN_MODE == "hip" and self.training and x.is_cuda:
            from ..ops.bn_nhwc import bn_act, supported

            if supported(x) and self.weight.dtype == torch.float32 and (
                    residual is None or (residual.dtype == x.dtype and residual.shape == x.shape)):
                return bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, residual, relu)
        y = self(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if relu else y


class _Conv(nn.Module):
    def __init__(self, cin, cout, k, stride=1, g=None):
        super().__init__()
        fan = cin * k * k
        self.weight = nn.Parameter(torch.randn(cout, cin, k, k, generator=g) * (2.0 / fan) ** 0.5)
        self.stride, self.pad = stride, k // 2

    def forward(self, x):
        return F.conv2d(x, self.weight.to(x.dtype), None, self.stride, self.pad)


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
        y = self.b1.act(self.c1(x))
        y = self.b2.act(self.c2(y))
        s = x if self.down is None else self.down[1].act(self.down[0](x), relu=False)
        return self.b3.act(self.c3(y), residual=s)


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

    def forward(self, x: torch.Tensor, compute_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """x: NHWC [B, H, W, 3] (or NCHW); returns log-probabilities (fp32)."""
        if x.dim() == 4 and x.shape[-1] == 3:
            x = x.permute(0, 3, 1, 2)
        cd = compute_dtype or x.dtype
        h = x.to(cd)
        if h.is_cuda:
            h = h.contiguous(memory_format=torch.channels_last)
        h = F.max_pool2d(self.stem_bn.act(self.stem(h)), 3, 2, 1)
        for b in self.blocks:
            h = b(h)
        # classifier in fp32 (2048 x 1000: negligible cost): bf16 logits of a
        # memorising synthetic run overflowed into NaN at lr 0.1
        h = h.float().mean((2, 3))
        return F.log_softmax(F.linear(h, self.fc_w, self.fc_b), dim=1)

    @staticmethod
    def loss(logp, target):
        return F.nll_loss(logp, target)


def resnet50(num_classes: int = 1000, seed: Optional[int] = 0) -> ResNet50:
    return ResNet50(num_classes, seed=seed)
