"""Checkpoint / resume with the reference's results layout.

The reference's tester declares ``Results/<save>/{Log.txt, ErrorRate.log,
Net, optState}`` (examples/EASGD_tester.lua:36-47; the server has the same
block commented out, examples/EASGD_server.lua:37-48) but never writes
``Net``/``optState``.  Here they are written:

* ``Net``      -- ``torch.save`` of the ordered list of parameter tensors in the
  reference's layout and walk order (``model.reference_state()`` when the model
  provides it, e.g. SpatialConvolutionMM weights as [Cout, Cin*k*k]); loadable
  with ``torch.load(..., weights_only=True)``.
* ``optState`` -- ``torch.save`` of a dict of tensors/numbers: step counters,
  ``stepsPerNode`` (AllReduceSGD), ``center`` (AllReduceEA / AsyncEA), the
  momentum buffer, learning rate, epoch and the BatchNorm running statistics.
* ``Log.txt`` / ``ErrorRate.log`` -- text logs (:class:`~torch_distlearn_amd.utils.metrics.Logger`).

Resume = :func:`load_checkpoint` on every node, then
``synchronizeParameters`` (root's values win, exactly like a fresh start).
Files are written by node 1 only, atomically (write to a temp name, rename).
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Optional

import torch

from .utils.walk import walk_table


def results_dir(save: str, root: str = "Results") -> str:
    d = os.path.join(root, save)
    os.makedirs(d, exist_ok=True)
    return d


def _atomic_save(obj, path: str) -> None:
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def _net_tensors(model_or_params) -> List[torch.Tensor]:
    if hasattr(model_or_params, "reference_state"):
        return [t.detach().cpu() for t in model_or_params.reference_state()]
    return [t.detach().cpu().clone() for t in walk_table(model_or_params)]


def save_checkpoint(directory: str, model_or_params: Any, opt_state: Optional[Dict[str, Any]] = None,
                    buffers: Optional[Dict[str, torch.Tensor]] = None) -> None:
    os.makedirs(directory, exist_ok=True)
    _atomic_save(_net_tensors(model_or_params), os.path.join(directory, "Net"))
    st: Dict[str, Any] = {}
    for k, v in (opt_state or {}).items():
        st[k] = v.detach().cpu().clone() if isinstance(v, torch.Tensor) else v
    if buffers is None and isinstance(model_or_params, torch.nn.Module):
        buffers = {n: b for n, b in model_or_params.named_buffers()}
    for n, b in (buffers or {}).items():
        st["buffer/" + n] = b.detach().cpu().clone()
    _atomic_save(st, os.path.join(directory, "optState"))


@torch.no_grad()
def load_checkpoint(directory: str, model_or_params: Any) -> Dict[str, Any]:
    """Load ``Net`` into the model/params (in place) and return ``optState``.
    Uses ``weights_only=True`` loads only."""
    net = torch.load(os.path.join(directory, "Net"), weights_only=True)
    if hasattr(model_or_params, "load_reference_state"):
        model_or_params.load_reference_state(net)
    else:
        leaves = walk_table(model_or_params)
        if len(leaves) != len(net):
            raise ValueError(f"checkpoint has {len(net)} tensors, model has {len(leaves)}")
        for t, v in zip(leaves, net):
            t.copy_(v.reshape(t.shape))
    st_path = os.path.join(directory, "optState")
    st = torch.load(st_path, weights_only=True) if os.path.exists(st_path) else {}
    if isinstance(model_or_params, torch.nn.Module):
        bufs = dict(model_or_params.named_buffers())
        for k, v in st.items():
            if k.startswith("buffer/") and k[7:] in bufs:
                bufs[k[7:]].copy_(v)
    return st


def trainer_state(trainer) -> Dict[str, Any]:
    """Collect the algorithm state of a DataParallelTrainer for ``optState``."""
    st: Dict[str, Any] = {"lr": trainer.lr, "steps": trainer.steps}
    if trainer.sgd is not None:
        st["stepsPerNode"] = trainer.sgd.stepsPerNode
    if trainer.ea is not None:
        st["center"] = trainer.ea.center
        st["ea_step"] = trainer.ea.step
    if trainer.mom is not None:
        st["momentum"] = trainer.mom
    return st


def restore_trainer_state(trainer, st: Dict[str, Any]) -> None:
    trainer.steps = int(st.get("steps", 0))
    if trainer.sgd is not None and "stepsPerNode" in st:
        trainer.sgd.stepsPerNode.copy_(st["stepsPerNode"])
    if trainer.ea is not None and "center" in st:
        trainer.ea.center.copy_(st["center"].to(trainer.ea.center.device))
        trainer.ea.step = int(st.get("ea_step", 0))
    if trainer.mom is not None and "momentum" in st:
        trainer.mom.copy_(st["momentum"].to(trainer.mom.device))
