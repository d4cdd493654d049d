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

Training resume (SURVEY §5.4 "resume = load + synchronizeParameters"):
:func:`save_trainer` is called by every node at an epoch boundary (after the
epoch-end synchronisation) and :func:`resume_trainer` on every node of the
restarted job.  optState then also carries ``stepsPerNode``, the EA ``center``
and ``ea_step``, the momentum buffer, lr, epoch and per-node counters (e.g.
batches drawn, so each node's sampler continues its stream); for AllReduceEA
every node's own parameters (and momentum) are gathered into optState too,
because elastic replicas differ between nodes.  Loading refreshes the bf16
shadow the HIP executor computes with, and the algorithm's resynchronisation
keeps what was restored: AllReduceSGD broadcasts node 1's (identical)
parameters, AllReduceEA runs ``synchronizeCenter`` (an idle drain + center
scatter), which leaves both the restored center and the local parameters in
place.  Result: a run resumed from epoch k is bitwise the run that never
stopped (tests/distributed/test_resume.py).

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
    """The algorithm state of a DataParallelTrainer for ``optState`` (node-local
    view; :func:`save_trainer` adds the per-node parts)."""
    return _trainer_state(trainer)


def _trainer_state(trainer) -> Dict[str, Any]:
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
    """Inverse of :func:`trainer_state` (node-local parts)."""
    trainer.steps = int(st.get("steps", 0))
    trainer.lr = float(st.get("lr", trainer.lr))
    if trainer.sgd is not None and "stepsPerNode" in st:
        trainer.sgd.stepsPerNode.copy_(st["stepsPerNode"])
    if trainer.ea is not None and "center" in st:
        trainer.ea.center.copy_(st["center"].to(trainer.ea.center.device))
        trainer.ea.step = int(st.get("ea_step", 0))
    if trainer.mom is not None and "momentum" in st:
        trainer.mom.copy_(st["momentum"].to(trainer.mom.device))


def _gather_rows(comm, t: torch.Tensor) -> torch.Tensor:
    """[world, numel] copy of every node's ``t`` (collective)."""
    out = torch.empty(comm.world_size * t.numel(), dtype=t.dtype, device=t.device)
    comm.all_gather(out, t.contiguous().view(-1))
    return out.view(comm.world_size, -1)


def save_trainer(directory: str, trainer, epoch: int, per_node: Optional[Dict[str, int]] = None,
                 extra: Optional[Dict[str, Any]] = None) -> None:
    """Checkpoint a :class:`~torch_distlearn_amd.engine.DataParallelTrainer`
    into ``directory`` (``Results/<save>``).  Collective: every node calls it
    at the same point (after the epoch-end synchronisation); node 1 writes
    ``Net`` and ``optState``.  ``per_node`` integers (e.g. batches drawn) are
    gathered into ``optState['node/<key>']`` = int64[numNodes]."""
    tree, flat = trainer.tree, trainer.flat
    comm = tree.comm
    st = _trainer_state(trainer)
    st["epoch"] = int(epoch)
    st["algo"] = trainer.algo
    for k, v in (per_node or {}).items():
        row = torch.zeros(tree.numNodes, dtype=torch.int64)
        row[tree.nodeIndex - 1] = int(v)
        comm.all_reduce_host(row, "sum")
        st["node/" + k] = row
    if trainer.algo == "ea":
        # elastic replicas differ between nodes: keep every node's own params (+ momentum)
        st["params_per_node"] = _gather_rows(comm, flat.data)
        if trainer.mom is not None:
            st["momentum_per_node"] = _gather_rows(comm, trainer.mom)
    st.update(extra or {})
    if tree.nodeIndex == 1:
        save_checkpoint(directory, trainer.model, st)
    comm.barrier()


def resume_trainer(directory: str, trainer) -> Dict[str, Any]:
    """Restore a trainer from :func:`save_trainer`'s files (every node), then
    resynchronise the way the algorithm needs (see the module docstring).
    Returns optState (``epoch``, ``node/<key>`` counters, ...)."""
    flat = trainer.flat
    st = load_checkpoint(directory, trainer.model)
    restore_trainer_state(trainer, st)
    me = trainer.tree.nodeIndex - 1
    with torch.no_grad():  # per-node parts override node 1's
        if "params_per_node" in st:
            flat.data.copy_(st["params_per_node"][me].to(flat.data.device))
        if "momentum_per_node" in st and trainer.mom is not None:
            trainer.mom.copy_(st["momentum_per_node"][me].to(trainer.mom.device))
    flat.refresh_shadow()  # the HIP executor computes with the bf16 shadow
    if trainer.algo == "sgd":
        trainer.sgd.synchronizeParameters(flat)
    elif trainer.algo == "ea":
        trainer.ea.synchronizeCenter(flat)  # step 0 everywhere: idle drain + center scatter
    return st
