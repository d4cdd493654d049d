"""The reference's CIFAR-10 convnet (examples/cifar10.lua:101-143,
examples/Model.lua:20-52): four blocks of

    conv 5x5/1 pad 2 -> SpatialBatchNormalization(C, eps=1e-3) -> ReLU -> maxpool 2x2/2

with 3->64->128->256->512 channels (32->16->8->4->2 spatial), then
Linear(512*2*2, 10) -> LogSoftMax -> ClassNLLCriterion.
4,328,970 parameters in 18 tensors (SURVEY §2.8 "P_c").

MI355X layout decisions (not the reference's):

* activations are NHWC (channels-last): the implicit-GEMM conv kernels read
  a (kh, kw, c) slice of K contiguously with 16-byte loads;
* conv weights are stored ``[Cout, 5, 5, Cin]`` (KRSC), i.e. already the
  [N][K] B-operand layout of the MFMA implicit GEMM;
* the linear layer consumes the NHWC flatten order (h, w, c).

``checkpoint.py`` converts to/from the reference layout (SpatialConvolutionMM
weight ``[Cout, Cin*5*5]`` in (c, kh, kw) order and NCHW flatten order for the
linear weight), so the ``Results/<save>/Net`` checkpoint stays compatible.

This module is the *torch* execution path (CPU / numerics reference / MIOpen
baseline).  The MI355X execution path with hand-written HIP kernels and a
hipGraph-captured step is :class:`torch_distlearn_amd.models.cifar_hip.CifarHIPExecutor`,
which runs on the *same* parameter tensors.
"""
from __future__ import annotations

import math
from typing import List, Sequence

import torch
import torch.nn as nn
import torch.nn.functional as F

CHANNELS = (3, 64, 128, 256, 512)
KSIZE = 5
PAD = 2
BN_EPS = 1e-3          # examples/cifar10.lua:109
BN_MOMENTUM = 0.1      # nn.SpatialBatchNormalization default
NUM_CLASSES = 10
IMAGE = 32


class CifarConvNet(nn.Module):
    """Parameters are registered in the reference's walk order:
    conv1.w, conv1.b, bn1.w, bn1.b, ..., conv4.b, bn4.w, bn4.b, fc.w, fc.b
    (params[1..9] of examples/cifar10.lua:108-133)."""

    def __init__(self, channels: Sequence[int] = CHANNELS, num_classes: int = NUM_CLASSES,
                 image: int = IMAGE, bn_eps: float = BN_EPS, seed: int | None = 0):
        super().__init__()
        self.channels = tuple(channels)
        self.nblocks = len(channels) - 1
        self.bn_eps = bn_eps
        self.num_classes = num_classes
        self.image = image
        self.final_hw = image >> self.nblocks
        g = torch.Generator().manual_seed(seed) if seed is not None else None  # same init on all nodes (:105)
        for i in range(self.nblocks):
            cin, cout = channels[i], channels[i + 1]
            fan_in = cin * KSIZE * KSIZE
            bound = 1.0 / math.sqrt(fan_in)  # nn.SpatialConvolutionMM:reset() (uniform +-1/sqrt(fan_in))
            w = (torch.rand(cout, KSIZE, KSIZE, cin, generator=g) * 2 - 1) * bound
            b = (torch.rand(cout, generator=g) * 2 - 1) * bound
            self.register_parameter(f"conv{i + 1}_w", nn.Parameter(w))
            self.register_parameter(f"conv{i + 1}_b", nn.Parameter(b))
            self.register_parameter(f"bn{i + 1}_w", nn.Parameter(torch.rand(cout, generator=g)))  # BN reset(): U(0,1)
            self.register_parameter(f"bn{i + 1}_b", nn.Parameter(torch.zeros(cout)))
            self.register_buffer(f"bn{i + 1}_rm", torch.zeros(cout))
            self.register_buffer(f"bn{i + 1}_rv", torch.ones(cout))
        feat = channels[-1] * self.final_hw * self.final_hw
        bound = 1.0 / math.sqrt(feat)
        self.fc_w = nn.Parameter((torch.rand(num_classes, feat, generator=g) * 2 - 1) * bound)
        self.fc_b = nn.Parameter((torch.rand(num_classes, generator=g) * 2 - 1) * bound)

    # ------------------------------------------------------------------
    def conv_w(self, i: int) -> torch.Tensor:
        return getattr(self, f"conv{i + 1}_w")

    def block_params(self, i: int):
        return (getattr(self, f"conv{i + 1}_w"), getattr(self, f"conv{i + 1}_b"), getattr(self, f"bn{i + 1}_w"),
                getattr(self, f"bn{i + 1}_b"), getattr(self, f"bn{i + 1}_rm"), getattr(self, f"bn{i + 1}_rv"))

    def forward(self, x: torch.Tensor, compute_dtype: torch.dtype | None = None) -> torch.Tensor:
        """x: NHWC [B, H, W, 3] (or NCHW [B, 3, H, W]); returns log-probabilities
        [B, num_classes] in fp32.  ``compute_dtype=torch.bfloat16`` runs convs
        and the linear layer in bf16 with fp32 BN statistics (the mixed
        precision the HIP path uses)."""
        if x.dim() == 4 and x.shape[-1] != self.channels[0] and x.shape[1] == self.channels[0]:
            x = x.permute(0, 2, 3, 1)
        cd = compute_dtype or x.dtype
        h = x.permute(0, 3, 1, 2).to(cd)  # logical NCHW view of NHWC storage
        if h.is_cuda:
            h = h.contiguous(memory_format=torch.channels_last)
        for i in range(self.nblocks):
            w, b, g, beta, rm, rv = self.block_params(i)
            wk = w.permute(0, 3, 1, 2).to(cd)  # KRSC -> KCRS view
            h = F.conv2d(h, wk, b.to(cd), stride=1, padding=PAD)
            h = F.batch_norm(h.float(), rm, rv, g, beta, self.training, BN_MOMENTUM, self.bn_eps).to(cd)
            h = F.max_pool2d(F.relu(h), 2, 2)
        h = h.permute(0, 2, 3, 1).reshape(h.shape[0], -1)  # NHWC flatten (h, w, c)
        logits = F.linear(h, self.fc_w.to(cd), self.fc_b.to(cd)).float()
        return F.log_softmax(logits, dim=1)

    @staticmethod
    def loss(logp: torch.Tensor, target: torch.Tensor) -> torch.Tensor:
        return F.nll_loss(logp, target)  # ClassNLLCriterion (mean)

    def param_list(self) -> List[torch.Tensor]:
        return list(self.parameters())

    # ---------------------------------------------------- reference layout I/O
    @torch.no_grad()
    def reference_state(self) -> List[torch.Tensor]:
        """Parameters in the reference's layout and walk order (the ``Net``
        checkpoint): SpatialConvolutionMM weights [Cout, Cin*5*5] in (c, kh, kw)
        order, the linear weight over the NCHW flatten (c, h, w)."""
        out = []
        for i in range(self.nblocks):
            w, b, g, beta, _, _ = self.block_params(i)
            out += [w.permute(0, 3, 1, 2).reshape(w.shape[0], -1).clone(), b.clone(), g.clone(), beta.clone()]
        C, hw = self.channels[-1], self.final_hw
        fw = self.fc_w.reshape(self.num_classes, hw, hw, C).permute(0, 3, 1, 2).reshape(self.num_classes, -1)
        return out + [fw.clone(), self.fc_b.clone()]

    @torch.no_grad()
    def load_reference_state(self, tensors: List[torch.Tensor]) -> None:
        it = iter(tensors)
        for i in range(self.nblocks):
            w, b, g, beta, _, _ = self.block_params(i)
            cout, k, _, cin = w.shape
            w.copy_(next(it).reshape(cout, cin, k, k).permute(0, 2, 3, 1))
            b.copy_(next(it))
            g.copy_(next(it))
            beta.copy_(next(it))
        C, hw = self.channels[-1], self.final_hw
        self.fc_w.copy_(next(it).reshape(self.num_classes, C, hw, hw).permute(0, 2, 3, 1).reshape(self.num_classes, -1))
        self.fc_b.copy_(next(it))


def num_params(model: nn.Module) -> int:
    return sum(p.numel() for p in model.parameters())
