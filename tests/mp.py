"""Multi-process harness: the reference spawned N-1 worker threads with
``ipc.map`` around a real TCP backend on 127.0.0.1 (test/test_AllReduceSGD.lua:
26-35); here N processes run on gloo over 127.0.0.1 with an ephemeral port."""
import os
import socket
import traceback

import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _to_host(x):
    """Tensors -> numpy (pickled by value; torch's shared-memory tensor
    pickling dies with the worker process)."""
    import torch

    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy().copy()
    if isinstance(x, (list, tuple)):
        return type(x)(_to_host(v) for v in x)
    if isinstance(x, dict):
        return {k: _to_host(v) for k, v in x.items()}
    return x


def _entry(rank, world, port, fn, args, q):
    os.environ["OMP_NUM_THREADS"] = "1"
    try:
        import torch

        torch.set_num_threads(1)
        res = _to_host(fn(rank, world, port, *args))
        q.put((rank, "ok", res))
    except Exception:  # pragma: no cover - reported to parent
        q.put((rank, "err", traceback.format_exc()))


def run(fn, world: int, *args, timeout: float = 240.0, dead=()):
    """Run ``fn(rank, world, port, *args)`` in ``world`` processes; return the
    per-rank results (raises on any worker failure or timeout).  Ranks in
    ``dead`` are expected to die without reporting (fault-injection tests):
    their result is None.  The ephemeral port is probed, then bound by rank 0's
    store a moment later; if another process took it in between (EADDRINUSE
    at rendezvous, seen once on a busy box) the whole run starts again on a
    fresh port, once."""
    try:
        return _run(fn, world, *args, timeout=timeout, dead=dead)
    except RuntimeError as e:
        if "EADDRINUSE" not in str(e):
            raise
        return _run(fn, world, *args, timeout=timeout, dead=dead)


def _run(fn, world: int, *args, timeout: float = 240.0, dead=()):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_entry, args=(r, world, port, fn, args, q), daemon=True) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    try:
        for _ in range(world - len(dead)):
            rank, status, payload = q.get(timeout=timeout)
            if status != "ok":
                raise RuntimeError(f"rank {rank} failed:\n{payload}")
            results[rank] = payload
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    return [results.get(r) for r in range(world)]
