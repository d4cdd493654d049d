"""Deterministic traversal of nested tensor tables.

Replaces ``ipc.utils.walkTable`` (used at lua/AllReduceSGD.lua:24,43,
lua/AllReduceEA.lua:16,35, lua/AsyncEA.lua:2-3).  Parameters and gradients in
the reference are arbitrary nested Lua tables of tensors (a dict in
examples/mnist.lua:56-66, a list of lists in examples/cifar10.lua:101-133).
The walk order must be identical on every node because AllReduceEA indexes
``center[i]`` by walk position (lua/AllReduceEA.lua:34-39), so dict keys are
visited in sorted order (not insertion order) here.
"""
from __future__ import annotations

from typing import Any, Callable, List

import torch


def _keys(d: dict):
    try:
        return sorted(d.keys())
    except TypeError:  # mixed key types: sort by (type name, repr)
        return sorted(d.keys(), key=lambda k: (type(k).__name__, repr(k)))


def walk_table(t: Any, fn: Callable[[torch.Tensor], Any] | None = None) -> List[torch.Tensor]:
    """Visit every tensor leaf of ``t`` in deterministic order.

    ``fn(tensor)`` is called for each leaf; if ``fn`` returns a tensor *and* the
    container is mutable, the leaf is replaced (like walkTable's return value).
    Returns the list of (possibly replaced) leaves in walk order.
    Accepts tensors, ``torch.nn.Module`` (its parameters, registration order),
    dicts, lists, tuples and ``None`` (no leaves).
    """
    out: List[torch.Tensor] = []

    def visit(node):
        if node is None:
            return None
        if isinstance(node, torch.Tensor):
            r = fn(node) if fn is not None else None
            leaf = r if isinstance(r, torch.Tensor) else node
            out.append(leaf)
            return leaf
        if isinstance(node, torch.nn.Module):
            for p in node.parameters():
                visit(p)
            return node
        if isinstance(node, dict):
            for k in _keys(node):
                v = node[k]
                nv = visit(v)
                if isinstance(v, torch.Tensor) and nv is not v:
                    node[k] = nv
            return node
        if isinstance(node, list):
            for i, v in enumerate(node):
                nv = visit(v)
                if isinstance(v, torch.Tensor) and nv is not v:
                    node[i] = nv
            return node
        if isinstance(node, tuple):
            for v in node:
                visit(v)
            return node
        if hasattr(node, "tensors") and callable(getattr(node, "tensors")):
            for v in node.tensors():
                visit(v)
            return node
        raise TypeError(f"walk_table: unsupported node type {type(node).__name__}")

    visit(t)
    return out


# reference spelling
walkTable = walk_table


def map_table(t: Any, fn: Callable[[torch.Tensor], torch.Tensor]) -> Any:
    """Structure-preserving map returning a *new* table (fn(leaf) per leaf)."""
    if t is None:
        return None
    if isinstance(t, torch.Tensor):
        return fn(t)
    if isinstance(t, dict):
        return {k: map_table(t[k], fn) for k in _keys(t)}
    if isinstance(t, list):
        return [map_table(v, fn) for v in t]
    if isinstance(t, tuple):
        return tuple(map_table(v, fn) for v in t)
    if isinstance(t, torch.nn.Module):
        return [fn(p) for p in t.parameters()]
    raise TypeError(f"map_table: unsupported node type {type(t).__name__}")


def clone_table(t: Any) -> Any:
    return map_table(t, lambda x: x.detach().clone())
