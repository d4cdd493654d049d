"""Metrics and logging.

* :class:`ConfusionMatrix` -- optim.ConfusionMatrix as used by the reference
  (``confusionMatrix:add(prediction[b], y[b])`` per sample,
  examples/cifar10.lua:194-196; all-reduced across nodes before printing,
  examples/cifar10.lua:203,234, examples/mnist.lua:119-125).  On the GPU the
  whole batch is accumulated by ONE HIP kernel (argmax by wave reduction +
  64-bit atomics, csrc/kernels/metrics.hip ``confusion_update``); the int64
  matrix is all-reduced with one collective (``allReduce(self)``).
* :class:`Logger` -- optim.Logger: a header of column names, then one
  tab-separated row per ``add`` (``Results/<save>/ErrorRate.log`` with
  "Training Error" / "Test Error", examples/EASGD_tester.lua:47,161-165).
* :class:`JsonlMetrics` -- machine-readable step metrics stream
  (step time, images/s, n, loss).
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, List, Optional, Sequence

import torch

from .._native import native, stream_handle


class ConfusionMatrix:
    def __init__(self, classes, device=None):
        if isinstance(classes, int):
            classes = [str(i + 1) for i in range(classes)]
        self.classes = list(classes)
        self.nclasses = len(self.classes)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self.mat = torch.zeros(self.nclasses, self.nclasses, dtype=torch.int64, device=self.device)

    def zero(self) -> None:
        self.mat.zero_()

    def add(self, prediction: torch.Tensor, target) -> None:
        """prediction: [C] or [B, C] scores/log-probs; target: int or [B]
        (0-based; the reference's 1-based labels are shifted by the loaders)."""
        pred = prediction if prediction.dim() == 2 else prediction.unsqueeze(0)
        tgt = torch.as_tensor(target, device=pred.device).reshape(-1).to(torch.int64)
        if pred.is_cuda:
            if self.mat.device != pred.device:
                self.mat = self.mat.to(pred.device)
            p = pred.contiguous()
            if p.dtype not in (torch.float32, torch.bfloat16):
                p = p.float()
            t = tgt.contiguous()
            native().confusion_update(p.data_ptr(), int(p.dtype == torch.bfloat16), t.data_ptr(), self.mat.data_ptr(),
                                      p.shape[0], self.nclasses, stream_handle())
            return
        am = pred.float().argmax(dim=1)
        idx = tgt.to(self.mat.device) * self.nclasses + am.to(self.mat.device)
        self.mat.view(-1).index_add_(0, idx, torch.ones_like(idx))

    batchAdd = add  # noqa: N815  (optim.ConfusionMatrix:batchAdd)

    def allReduce(self, tree) -> None:  # noqa: N802
        """Sum the matrix over all nodes (``tree.allReduce(confusionMatrix.mat, add)``)."""
        tree.allReduce([self.mat], "sum")

    @property
    def totalValid(self) -> float:  # noqa: N802
        tot = int(self.mat.sum())
        return float(self.mat.diagonal().sum()) / tot if tot else 0.0

    @property
    def averageValid(self) -> float:  # noqa: N802
        m = self.mat.double()
        rows = m.sum(1)
        valid = rows > 0
        return float((m.diagonal()[valid] / rows[valid]).mean()) if bool(valid.any()) else 0.0

    def __str__(self) -> str:
        m = self.mat.cpu()
        lines = ["ConfusionMatrix:"]
        for i in range(self.nclasses):
            row = " ".join(f"{int(v):6d}" for v in m[i])
            tot = int(m[i].sum())
            acc = 100.0 * int(m[i, i]) / tot if tot else 0.0
            br = ("[[" if i == 0 else " [") + row + ("]]" if i == self.nclasses - 1 else "]")
            lines.append(f"{br}   {acc:7.3f}% \t[class: {self.classes[i]}]")
        lines.append(f" + average row correct: {100 * self.averageValid:.3f}% ")
        lines.append(f" + global correct: {100 * self.totalValid:.3f}%")
        return "\n".join(lines)


class Logger:
    """optim.Logger(path): ``setNames(names)`` then ``add({name = value})``."""

    def __init__(self, path: str, names: Optional[Sequence[str]] = None):
        self.path = path
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        self.names: List[str] = []
        self._f = open(path, "w")
        if names:
            self.setNames(names)

    def setNames(self, names: Sequence[str]) -> None:  # noqa: N802
        self.names = list(names)
        self._f.write("\t".join(self.names) + "\n")
        self._f.flush()

    def add(self, values: Dict[str, float]) -> None:
        if not self.names:
            self.setNames(sorted(values))
        self._f.write("\t".join(f"{float(values[n]):.4e}" for n in self.names) + "\n")
        self._f.flush()

    def close(self) -> None:
        self._f.close()


class JsonlMetrics:
    """One JSON object per line; ``rank0_only`` mirrors the reference silencing
    non-root output (examples/cifar10.lua:30-33)."""

    def __init__(self, path: Optional[str], rank: int = 0, rank0_only: bool = True):
        self.enabled = path is not None and (rank == 0 or not rank0_only)
        self._f = open(path, "a") if self.enabled else None
        self.rank = rank
        self._t = time.perf_counter()

    def log(self, **kw) -> None:
        if not self.enabled:
            return
        kw.setdefault("rank", self.rank)
        kw.setdefault("t", round(time.perf_counter() - self._t, 6))
        self._f.write(json.dumps(kw) + "\n")
        self._f.flush()

    def close(self) -> None:
        if self._f:
            self._f.close()
