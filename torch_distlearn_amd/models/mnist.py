"""MNIST models.

* :class:`MnistConvNet` -- the reference's network (examples/mnist.lua:53-66,
  examples/mnist-ea.lua:41-57): Reshape(1,32,32) -> SpatialConvolutionMM(1,16,5,5)
  -> Tanh -> SpatialMaxPooling(2,2,2,2) -> SpatialConvolutionMM(16,16,5,5) ->
  Tanh -> SpatialMaxPooling(2,2,2,2) -> Reshape(16*5*5) -> Linear(400,10) ->
  util.logSoftMax, loss = logMultinomialLoss (examples/mnist.lua:75-88).
  10,842 parameters in 6 tensors (SURVEY §2.8 "P_m").
* :class:`MnistMLP` -- the 2-layer MLP of BASELINE.json config 1 (plumbing
  config, CPU/gloo): 1024 -> hidden -> 10.

Both are latency-bound (43 KB of parameters); on the GPU they run through
PyTorch ops inside a captured hipGraph (the engine's ``graph=True``), which is
what matters at this size.
"""
from __future__ import annotations

import math
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F


def _uniform(shape, bound, g):
    return (torch.rand(*shape, generator=g) * 2 - 1) * bound


class MnistConvNet(nn.Module):
    def __init__(self, seed: Optional[int] = 0, image: int = 32):
        super().__init__()
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        b1 = 1 / math.sqrt(1 * 25)
        b2 = 1 / math.sqrt(16 * 25)
        self.image = image
        feat = 16 * (((image - 4) // 2 - 4) // 2) ** 2
        b3 = 1 / math.sqrt(feat)
        # registration order == reference table order after walkTable's sorted keys:
        # conv1 {w, b}, conv2 {w, b}, linear {w, b}
        self.conv1_w = nn.Parameter(_uniform((16, 1, 5, 5), b1, g))
        self.conv1_b = nn.Parameter(_uniform((16,), b1, g))
        self.conv2_w = nn.Parameter(_uniform((16, 16, 5, 5), b2, g))
        self.conv2_b = nn.Parameter(_uniform((16,), b2, g))
        self.fc_w = nn.Parameter(_uniform((10, feat), b3, g))
        self.fc_b = nn.Parameter(_uniform((10,), b3, g))

    def forward(self, x: torch.Tensor, compute_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        """x: [B, 1024] / [B, 32, 32] / [B, 32, 32, 1] / [B, 1, 32, 32]."""
        B = x.shape[0]
        cd = compute_dtype or (x.dtype if x.is_floating_point() else torch.float32)
        h = x.reshape(B, 1, self.image, self.image).to(cd)
        h = F.max_pool2d(torch.tanh(F.conv2d(h, self.conv1_w.to(cd), self.conv1_b.to(cd))), 2, 2)
        h = F.max_pool2d(torch.tanh(F.conv2d(h, self.conv2_w.to(cd), self.conv2_b.to(cd))), 2, 2)
        h = h.reshape(B, -1)
        return F.log_softmax(F.linear(h, self.fc_w.to(cd), self.fc_b.to(cd)).float(), dim=1)

    @staticmethod
    def loss(logp: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        # logMultinomialLoss with one-hot targets == NLL of the log-probabilities
        return F.nll_loss(logp, target)


class MnistMLP(nn.Module):
    def __init__(self, in_dim: int = 1024, hidden: int = 128, classes: int = 10, seed: Optional[int] = 0):
        super().__init__()
        g = torch.Generator().manual_seed(seed) if seed is not None else None
        b1, b2 = 1 / math.sqrt(in_dim), 1 / math.sqrt(hidden)
        self.in_dim = in_dim
        self.fc1_w = nn.Parameter(_uniform((hidden, in_dim), b1, g))
        self.fc1_b = nn.Parameter(_uniform((hidden,), b1, g))
        self.fc2_w = nn.Parameter(_uniform((classes, hidden), b2, g))
        self.fc2_b = nn.Parameter(_uniform((classes,), b2, g))

    def forward(self, x: torch.Tensor, compute_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
        B = x.shape[0]
        cd = compute_dtype or (x.dtype if x.is_floating_point() else torch.float32)
        h = torch.tanh(F.linear(x.reshape(B, -1).to(cd), self.fc1_w.to(cd), self.fc1_b.to(cd)))
        return F.log_softmax(F.linear(h, self.fc2_w.to(cd), self.fc2_b.to(cd)).float(), dim=1)

    @staticmethod
    def loss(logp: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return F.nll_loss(logp, target)
