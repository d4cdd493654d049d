"""Loader for the in-tree native library ``torch_distlearn_amd._C``.

The extension holds every hand-written gfx950 HIP kernel, the RCCL
communicator and the C++ data runtime.  It is built in-tree by
``csrc/build.py`` (``__graft_entry__.build()``).  GPU code paths call
:func:`native` which raises loudly if the library is missing -- there is no
silent eager/PyTorch fallback for GPU tensors.  CPU tensors (gloo tests) use
plain torch ops, which is a different device path, not a fallback.
"""
from __future__ import annotations

import importlib
import os

import torch  # noqa: F401  (must be loaded first: _C binds to torch's HIP runtime + RCCL)

_C = None
_ERR: Exception | None = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    try:
        _C = importlib.import_module("torch_distlearn_amd._C")
    except Exception as e:  # pragma: no cover - depends on build state
        if os.environ.get("DISTLEARN_AUTOBUILD", "0") == "1":
            from importlib import util as _u
            import sys

            root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
            sys.path.insert(0, os.path.join(root, "csrc"))
            spec = _u.spec_from_file_location("_dl_build", os.path.join(root, "csrc", "build.py"))
            mod = _u.module_from_spec(spec)
            spec.loader.exec_module(mod)
            mod.build()
            _C = importlib.import_module("torch_distlearn_amd._C")
        else:
            _ERR = e


def available() -> bool:
    _load()
    return _C is not None


def native():
    """Return the native module or raise (used by every GPU code path)."""
    _load()
    if _C is None:
        raise RuntimeError(
            "torch_distlearn_amd native library (_C) is not built/loadable; run "
            "`python csrc/build.py` (or __graft_entry__.build()). Original error: %r" % (_ERR,))
    return _C


def testing():
    """The test/diagnostic extension ``_C_testing`` (csrc/testing/: CU-occupancy
    spin kernels for the watchdog test and the RCCL footprint emulation).  It is
    deliberately not part of the product library ``_C``."""
    native()
    return importlib.import_module("torch_distlearn_amd._C_testing")


def stream_handle(stream=None) -> int:
    """Raw HIP stream handle of a torch stream (default: current stream)."""
    if stream is None:
        stream = torch.cuda.current_stream()
    return int(stream.cuda_stream)
