"""Local multi-process launcher + the reference's common CLI flags.

Reference launchers fork N ``th`` processes with ``--nodeIndex i --numNodes N``
and ``&``/``wait`` (examples/mnist.sh:4-10, examples/cifar10-cuda.sh:4-10,
examples/AsyncEASGD.sh:36-57).  Here::

    python -m torch_distlearn_amd.launch --nproc 4 examples/mnist.py [args...]

starts 4 child processes (never ``exec``: each is a fresh interpreter), passes
``--nodeIndex i --numNodes N`` (1-based, like the reference) plus the
torch.distributed environment (RANK / WORLD_SIZE / LOCAL_RANK / MASTER_ADDR /
MASTER_PORT on 127.0.0.1), streams their output, and returns the first
non-zero exit code.  ``--gpus`` assigns one GPU per node (``--gpu i``, the
reference's 1-based ``cutorch.setDevice``).  Scripts started by
``torch.distributed.run`` work too: :func:`node_opts` falls back to the env.
"""
from __future__ import annotations

import argparse
import os
import socket
import subprocess
import sys
from typing import List, Optional


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def add_node_flags(ap: argparse.ArgumentParser, batch: int = 32, lr: float = 0.1) -> argparse.ArgumentParser:
    """The flag block shared by the reference's scripts."""
    ap.add_argument("--nodeIndex", type=int, default=None, help="1-based node index (default: $RANK+1 or 1)")
    ap.add_argument("--numNodes", type=int, default=None, help="number of nodes (default: $WORLD_SIZE or 1)")
    ap.add_argument("--batchSize", type=int, default=batch)
    ap.add_argument("--learningRate", type=float, default=lr)
    ap.add_argument("--cuda", action="store_true", help="run on the GPU")
    ap.add_argument("--gpu", type=int, default=None, help="1-based GPU index (default: node-local rank + 1)")
    ap.add_argument("--host", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("MASTER_PORT", "8080")))
    ap.add_argument("--base", type=int, default=2, help="tree arity (accepted for parity; RCCL picks rings/trees)")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--commTimeout", type=float, default=None,
                    help="seconds before a dead/stuck peer turns into an error (default 600; DISTLEARN_COMM_TIMEOUT). "
                         "AsyncEA: the server's wait for the next client sync is bounded by it, so it must exceed "
                         "tau training steps of the slowest client; the tester's wait for its next snapshot is "
                         "unbounded (a dead server fails it at once)")
    return ap


def add_checkpoint_flags(ap: argparse.ArgumentParser) -> argparse.ArgumentParser:
    """``--save NAME`` writes Results/NAME/{Net, optState} after every epoch;
    ``--resume`` continues from them."""
    ap.add_argument("--save", default=None, help="checkpoint directory name under --resultsRoot")
    ap.add_argument("--resultsRoot", default="Results")
    ap.add_argument("--resume", action="store_true", help="resume from Results/<save>")
    return ap


def node_opts(opt) -> None:
    """Fill nodeIndex/numNodes/gpu from torchrun-style env when not given;
    export ``--commTimeout`` for the communicators."""
    if getattr(opt, "commTimeout", None) is not None:
        os.environ["DISTLEARN_COMM_TIMEOUT"] = str(opt.commTimeout)
    if opt.nodeIndex is None:
        opt.nodeIndex = int(os.environ.get("RANK", "0")) + 1
    if opt.numNodes is None:
        opt.numNodes = int(os.environ.get("WORLD_SIZE", "1"))
    if getattr(opt, "gpu", None) is None:
        opt.gpu = int(os.environ.get("LOCAL_RANK", str(opt.nodeIndex - 1))) + 1


def device_of(opt):
    import torch

    if getattr(opt, "cuda", False):
        n = torch.cuda.device_count()
        idx = (opt.gpu - 1) % max(1, n)
        torch.cuda.set_device(idx)
        return torch.device("cuda", idx)
    return torch.device("cpu")


def quiet_unless_root(node_index: int) -> None:
    """Non-root nodes silence their output (examples/cifar10.lua:30-33)."""
    if node_index != 1:
        sys.stdout = open(os.devnull, "w")


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--nproc", type=int, required=True, help="number of local nodes (processes)")
    ap.add_argument("--gpus", action="store_true", help="give node i the GPU i (adds --cuda --gpu i)")
    ap.add_argument("--port", type=int, default=None, help="rendezvous port (default: a free port)")
    ap.add_argument("--no-node-flags", action="store_true", help="do not append --nodeIndex/--numNodes")
    ap.add_argument("script")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    port = a.port or free_port()
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    procs = []
    for i in range(a.nproc):
        env = dict(os.environ)
        env.update(RANK=str(i), LOCAL_RANK=str(i), WORLD_SIZE=str(a.nproc), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        cmd = [sys.executable, a.script] + list(a.args)
        if not a.no_node_flags:
            cmd += ["--nodeIndex", str(i + 1), "--numNodes", str(a.nproc), "--port", str(port)]
        if a.gpus:
            cmd += ["--cuda", "--gpu", str(i + 1)]
        procs.append(subprocess.Popen(cmd, env=env))
    rc = 0
    for p in procs:
        r = p.wait()
        if r != 0 and rc == 0:
            rc = r
    return rc


if __name__ == "__main__":
    sys.exit(main())
