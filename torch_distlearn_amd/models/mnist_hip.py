"""Native executor for the reference MNIST convnet: the whole forward +
backward of a training step is four small hand-written gfx950 kernels
(csrc/kernels/mnist.hip), each parallel over (channel x sample) workgroups.

Reference: examples/mnist.lua:53-130 (batch 1 per node, lr 0.01).  The
reference's step is ~35 library kernels for ~6 MFLOP of work, i.e. pure launch
latency; here it is these kernels + the engine's zero-fill
of the gradient buffer + the fused SGD update, all captured in one hipGraph
(``DataParallelTrainer(graph=True)``), with the whole 43 KB gradient in one
all-reduce bucket.
"""
from __future__ import annotations

from typing import Optional

import torch

from .._native import native, stream_handle
from .mnist import MnistConvNet


class MnistHIPExecutor:
    takes_loader = False      # batches come as tensors (the engine draws them from a loader)
    overwrites_grads = False  # gradients are atomically accumulated: the engine zero-fills them per step

    def __init__(self, model: MnistConvNet, flat, bucketer=None, max_batch: Optional[int] = None):
        if not isinstance(model, MnistConvNet) or model.image != 32:
            raise TypeError("MnistHIPExecutor needs the 32x32 MnistConvNet")
        if flat.data.dtype != torch.float32:
            raise ValueError("MnistHIPExecutor needs fp32 master parameters")
        self.C = native()
        self.model, self.flat, self.bucketer = model, flat, bucketer
        self.p = flat.param_views()   # conv1_w, conv1_b, conv2_w, conv2_b, fc_w, fc_b
        self.g = flat.views_of(flat.grad)
        dev = flat.data.device
        self.cap = int(max_batch or 1)
        self.logp = torch.empty(self.cap, 10, device=dev)
        self.loss_b = torch.empty(self.cap, device=dev)
        # per-sample activations / argmax bytes / conv2 output gradient (kernel scratch)
        self.scratch = torch.empty(self.C.mnist_scratch_bytes(self.cap) // 4, device=dev)
        self._last_b = 0

    def _input(self, x: torch.Tensor) -> torch.Tensor:
        B = x.shape[0]
        if B > self.cap:
            raise ValueError(f"batch {B} > executor capacity {self.cap}")
        if x.numel() != B * 1024:
            raise ValueError("MnistHIPExecutor expects [B, 1024] / [B, 32, 32] / [B, 32, 32, 1] inputs")
        if x.dtype not in (torch.bfloat16, torch.float32):
            x = x.float()
        return x.contiguous()

    def _launch(self, x: torch.Tensor, labels: Optional[torch.Tensor]):
        x = self._input(x)
        B = x.shape[0]
        p, g = self.p, self.g
        train = labels is not None
        self.C.mnist_step(x.data_ptr(), int(x.dtype == torch.bfloat16), labels.data_ptr() if train else 0,
                          *[t.data_ptr() for t in p], *[t.data_ptr() for t in g], self.logp.data_ptr(),
                          self.loss_b.data_ptr() if train else 0, self.scratch.data_ptr(), B, stream_handle())
        self._last_b = B
        return B

    def forward_backward(self, x, labels: torch.Tensor) -> torch.Tensor:
        if labels.dtype != torch.int64:
            raise ValueError("labels must be int64")
        B = self._launch(x, labels)
        if self.bucketer is not None:  # every gradient is final when the kernel ends
            for i in range(len(self.p)):
                self.bucketer.mark_leaf_ready(i)
        return self.loss_b[:B].mean()

    def last_logits(self) -> torch.Tensor:
        return self.logp[:self._last_b]

    @torch.no_grad()
    def predict(self, x: torch.Tensor, batch_stats: bool = False) -> torch.Tensor:
        """Log-probabilities of ``x``.  The MNIST net has no BatchNorm, so
        ``batch_stats`` (the trainer's train-mode-statistics flag) changes
        nothing; it is accepted so ``DataParallelTrainer.predict`` works on
        every executor."""
        B = self._launch(x, None)
        return self.logp[:B].clone()
