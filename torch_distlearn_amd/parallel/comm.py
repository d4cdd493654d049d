"""Communicators: the data plane and control plane under ``Tree``.

Reference transport: ``libipc`` TCP sockets + an unpipelined b-ary tree
(``ipc.Tree``).  MI355X design:

* **Data plane** -- :class:`RcclCommunicator`: the native C++ RCCL
  communicator (``csrc/comm/communicator.h``).  Collectives are enqueued on a
  caller-chosen HIP stream (default: torch's current stream), never block the
  host, and are legal inside hipGraph capture.  RCCL picks ring/tree channels
  over the 7 xGMI links per GPU.
* **Control plane** -- a gloo process group over the c10d TCPStore:
  rendezvous, the ncclUniqueId exchange, any-source receives (AsyncEA's mutex,
  which RCCL cannot express), small host-side reductions, and the whole CPU
  test path.
* :class:`ProcessGroupCommunicator` implements the same interface on a
  ``torch.distributed`` group (gloo on CPU -- used by the multi-process tests --
  or torch's own NCCL/RCCL group when ``backend='nccl'`` is requested).
"""
from __future__ import annotations

import contextlib
import datetime
import os
from typing import List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

from .._native import native, stream_handle

DTYPE_CODES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.int64: 3,
               torch.int32: 4, torch.uint8: 5, torch.float64: 6}
OP_CODES = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}
_DIST_OPS = {"sum": dist.ReduceOp.SUM, "prod": dist.ReduceOp.PRODUCT, "max": dist.ReduceOp.MAX,
             "min": dist.ReduceOp.MIN}

MSG_LEN = 8  # control-plane message = int64[MSG_LEN]

DEFAULT_TIMEOUT_S = 600.0


def comm_timeout(default: float = DEFAULT_TIMEOUT_S) -> float:
    """Communication timeout in seconds (``DISTLEARN_COMM_TIMEOUT``; the
    examples' ``--commTimeout`` flag sets it): control-plane (gloo) operations
    and the RCCL watchdog give up after this long instead of hanging on a dead
    or stuck peer."""
    v = os.environ.get("DISTLEARN_COMM_TIMEOUT")
    return float(v) if v not in (None, "") else default


class CommError(RuntimeError):
    """A collective or control-plane message could not complete: a peer died,
    hung past the timeout, or the transport failed.  The communicator is no
    longer usable."""


# collective-sequence tracking (DISTLEARN_DEBUG_SYNC=1): every data-plane
# collective a rank issues is folded into a running 64-bit FNV-1a hash of
# (op, dtype, count, op / root); see Communicator.seq_*
SEQ_KINDS = {"all_reduce": 1, "broadcast": 2, "all_gather": 3, "reduce_scatter": 4}
_FNV_OFFSET, _FNV_PRIME, _M64 = 0xCBF29CE484222325, 0x100000001B3, (1 << 64) - 1


def seq_tracking() -> bool:
    return os.environ.get("DISTLEARN_DEBUG_SYNC", "0") == "1"


class Communicator:
    """Interface shared by the RCCL and process-group communicators."""

    rank: int
    world_size: int
    ctrl: Optional[dist.ProcessGroup]
    # collective-sequence state (class defaults; per instance once written)
    _seq_h = _FNV_OFFSET
    _seq_n = 0
    _seq_rec: Optional[list] = None

    # ---------------- collective-sequence tracking ----------------
    # RCCL hangs -- it does not fail -- when ranks issue different collective
    # sequences (the likely failure of uneven epochs with unrolled hipGraphs and
    # drains).  With DISTLEARN_DEBUG_SYNC=1 each rank hashes every collective it
    # issues; a hipGraph capture RECORDS its collectives (seq_record) and every
    # replay folds that record in (seq_replay), so the hash follows what ran.
    # The algorithms compare the hashes over the control plane at their epoch
    # synchronisation (utils/debug.check_collective_sequence) and raise
    # CommError naming the ranks that differ.  Point-to-point traffic (AsyncEA)
    # is asymmetric by design and not hashed.
    def _note(self, kind: str, t: torch.Tensor, arg: int = 0) -> None:
        if not seq_tracking():
            return
        item = (SEQ_KINDS[kind], DTYPE_CODES.get(t.dtype, 99), int(t.numel()), int(arg))
        if self._seq_rec is not None:  # inside a capture: it runs at every replay
            self._seq_rec.append(item)
        else:
            self._seq_fold((item,))

    def _seq_fold(self, items) -> None:
        h = self._seq_h
        for it in items:
            for v in it:
                h = ((h ^ (v & _M64)) * _FNV_PRIME) & _M64
        self._seq_h = h
        self._seq_n += len(items)

    @contextlib.contextmanager
    def seq_record(self):
        """Record (instead of count) the collectives issued inside the block --
        a hipGraph capture; yields the list to hand to :meth:`seq_replay`."""
        prev, rec = self._seq_rec, []
        self._seq_rec = rec
        try:
            yield rec
        finally:
            self._seq_rec = prev

    def seq_replay(self, rec: Optional[list], times: int = 1) -> None:
        """Count a recorded sequence as issued ``times`` times (graph replays)."""
        if rec:
            for _ in range(times):
                self._seq_fold(rec)

    def seq_state(self) -> Tuple[int, int]:
        """(hash, number of collectives) of what this rank issued so far."""
        return self._seq_h, self._seq_n

    # ---------------- data plane (in-place, stream ordered) ----------------
    def all_reduce(self, t: torch.Tensor, op: str = "sum", stream=None) -> None:
        raise NotImplementedError

    def broadcast(self, t: torch.Tensor, root: int = 0, stream=None) -> None:
        raise NotImplementedError

    def all_gather(self, out: torch.Tensor, t: torch.Tensor, stream=None) -> None:
        """out = cat over ranks of t (out.numel() == world * t.numel())."""
        raise NotImplementedError

    def send(self, t: torch.Tensor, peer: int, stream=None) -> None:
        raise NotImplementedError

    def recv(self, t: torch.Tensor, peer: int, stream=None) -> None:
        raise NotImplementedError

    @contextlib.contextmanager
    def group(self):
        yield

    # ---------------- control plane (host, gloo) ----------------
    def barrier(self) -> None:
        if self.world_size > 1:
            with _ctrl_errors("barrier"):
                dist.barrier(group=self.ctrl)

    def send_msg(self, msg: Sequence[int], dst: int, tag: int = 0) -> None:
        buf = torch.zeros(MSG_LEN, dtype=torch.int64)
        buf[: len(msg)] = torch.tensor(list(msg), dtype=torch.int64)
        with _ctrl_errors(f"send to rank {dst}"):
            dist.send(buf, dst=dst, group=self.ctrl, tag=tag)

    def recv_msg(self, src: Optional[int] = None, tag: int = 0,
                 timeout: Optional[float] = None, unbounded: bool = False) -> Tuple[int, List[int]]:
        """Receive a control message; ``src=None`` = any source (recvAny).
        ``timeout`` (seconds) bounds the wait; default: the group's timeout;
        ``unbounded``: no time limit (a peer that dies still fails the wait:
        its connection closes)."""
        buf = torch.zeros(MSG_LEN, dtype=torch.int64)
        what = "receive from " + ("any rank" if src is None else f"rank {src}")
        with _ctrl_errors(what):
            if unbounded:
                work = (dist.irecv(buf, src=src, group=self.ctrl, tag=tag) if src is not None
                        else self.ctrl.recv_anysource([buf], tag))
                work.wait(datetime.timedelta(days=365))
                sender = src if src is not None else work._source_rank()
            elif timeout is None:
                sender = dist.recv(buf, src=src, group=self.ctrl, tag=tag)
            else:
                work = (dist.irecv(buf, src=src, group=self.ctrl, tag=tag) if src is not None
                        else self.ctrl.recv_anysource([buf], tag))
                if not work.wait(datetime.timedelta(seconds=timeout)):
                    raise CommError(f"{what}: nothing within {timeout:.1f} s")
                sender = src if src is not None else work._source_rank()
        return int(sender), buf.tolist()

    def all_reduce_host(self, t: torch.Tensor, op: str = "sum") -> None:
        """Small CPU all-reduce on the control plane."""
        if self.world_size > 1:
            with _ctrl_errors("host all-reduce"):
                dist.all_reduce(t, op=_DIST_OPS[op], group=self.ctrl)

    def all_gather_host(self, t: torch.Tensor) -> List[torch.Tensor]:
        """Small CPU all-gather on the control plane: every rank's ``t``."""
        if self.world_size == 1:
            return [t.clone()]
        out = [torch.empty_like(t) for _ in range(self.world_size)]
        with _ctrl_errors("host all-gather"):
            dist.all_gather(out, t, group=self.ctrl)
        return out

    def broadcast_object(self, obj, root: int = 0):
        lst = [obj]
        if self.world_size > 1:
            dist.broadcast_object_list(lst, src=root, group=self.ctrl)
        return lst[0]

    def health(self) -> str:
        return ""

    def check(self) -> None:
        """Raise :class:`CommError` if the communicator has failed."""
        h = self.health()
        if h:
            raise CommError(h)

    def close(self) -> None:
        pass


@contextlib.contextmanager
def _ctrl_errors(what: str):
    """gloo failures (peer closed the connection, op timed out) -> CommError."""
    try:
        yield
    except CommError:
        raise
    except RuntimeError as e:
        raise CommError(f"control plane: {what} failed: {e}") from e


class ProcessGroupCommunicator(Communicator):
    """Communicator over a torch.distributed group (gloo CPU or torch NCCL)."""

    def __init__(self, data_group=None, ctrl_group=None):
        self.data = data_group
        self.ctrl = ctrl_group if ctrl_group is not None else data_group
        self.rank = dist.get_rank(self.data) if dist.is_initialized() else 0
        self.world_size = dist.get_world_size(self.data) if dist.is_initialized() else 1
        self._ops = None  # pending p2p ops inside group()
        self._unstage = []

    def all_reduce(self, t, op="sum", stream=None):
        self._note("all_reduce", t, OP_CODES[op])
        if self.world_size == 1:
            return
        with _ctrl_errors("all-reduce"):
            if op == "avg":
                dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.data)
                t.div_(self.world_size)
            else:
                dist.all_reduce(t, op=_DIST_OPS[op], group=self.data)

    def broadcast(self, t, root=0, stream=None):
        self._note("broadcast", t, root)
        if self.world_size > 1:
            with _ctrl_errors("broadcast"):
                dist.broadcast(t, src=root, group=self.data)

    def all_gather(self, out, t, stream=None):
        self._note("all_gather", t)
        if self.world_size == 1:
            out.view(-1).copy_(t.view(-1))
            return
        with _ctrl_errors("all-gather"):
            if self._stage(t):  # gloo: host-staged for device tensors
                o = torch.empty(out.numel(), dtype=out.dtype)
                dist.all_gather_into_tensor(o, t.detach().reshape(-1).cpu(), group=self.data)
                out.view(-1).copy_(o)
            else:
                dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1), group=self.data)

    def _stage(self, t) -> bool:
        return t.is_cuda and dist.get_backend(self.data) == "gloo"

    def send(self, t, peer, stream=None):
        src = t.detach().cpu() if self._stage(t) else t
        if self._ops is not None:
            self._ops.append(dist.P2POp(dist.isend, src, peer, group=self.data))
            return
        with _ctrl_errors(f"send to rank {peer}"):
            dist.send(src, dst=peer, group=self.data)

    def recv(self, t, peer, stream=None):
        dst = torch.empty(t.shape, dtype=t.dtype) if self._stage(t) else t
        if self._ops is not None:
            self._ops.append(dist.P2POp(dist.irecv, dst, peer, group=self.data))
            if dst is not t:
                self._unstage.append((t, dst))
            return
        with _ctrl_errors(f"receive from rank {peer}"):
            dist.recv(dst, src=peer, group=self.data)
        if dst is not t:
            t.copy_(dst)

    @contextlib.contextmanager
    def group(self):
        """Point-to-point calls inside the block are issued together
        (``batch_isend_irecv``), so a ring of sends and receives cannot
        deadlock -- the gloo analogue of ncclGroupStart/End."""
        if self._ops is not None:  # nested: the outermost group issues
            yield
            return
        self._ops, self._unstage = [], []
        try:
            yield
            ops, unstage = self._ops, self._unstage
        finally:
            self._ops = None
        if ops:
            with _ctrl_errors("grouped send/recv"):
                for w in dist.batch_isend_irecv(ops):
                    w.wait()
        for t, h in unstage:
            t.copy_(h)


# CU footprint of RCCL's collectives: one workgroup per channel (rcclGenericKernel:
# 256 threads, ~280 registers/wave, 19.7 KiB LDS).  Compute kernels that do not fit
# beside it (here: the 128x128 wgrad, 141 registers/wave, and the 3-stage streaming
# conv) lose that CU for the collective's lifetime, and a grid sized to the whole chip
# then needs a second round (measured per kernel with scripts/emulate_rccl.py and
# bench_conv.py --occupy).  More channels move a bucket faster over the 7 xGMI
# links; fewer leave more CUs to the backward it overlaps.  The cap is therefore a
# per-communicator setting (ncclConfig_t::maxCTAs, csrc/comm/communicator.h) that
# the trainer MEASURES: DataParallelTrainer.select_policy times the step with every
# candidate cap (DISTLEARN_CHANNEL_CAPS, default 16 and 32) x overlap policy at
# world > 1 and keeps the fastest slowest-rank one.  A user's NCCL_MAX_NCHANNELS
# (process-wide, read by RCCL at init) still applies on top and pins the cap.
DEFAULT_RCCL_CHANNELS = 32
DEFAULT_CHANNEL_CAPS = (16, 32)


def rccl_channel_cap() -> int:
    """The cap a new communicator starts with (NCCL_MAX_NCHANNELS if the user
    set it, else DISTLEARN_CHANNEL_CAP, else 32)."""
    return int(os.environ.get("NCCL_MAX_NCHANNELS", os.environ.get("DISTLEARN_CHANNEL_CAP", DEFAULT_RCCL_CHANNELS)))


def channel_cap_candidates() -> List[int]:
    """The channel caps select_policy measures (one only when the user pinned
    NCCL_MAX_NCHANNELS / DISTLEARN_CHANNEL_CAP)."""
    if "NCCL_MAX_NCHANNELS" in os.environ or "DISTLEARN_CHANNEL_CAP" in os.environ:
        return [rccl_channel_cap()]
    v = os.environ.get("DISTLEARN_CHANNEL_CAPS")
    caps = [int(c) for c in v.split(",") if c.strip()] if v else list(DEFAULT_CHANNEL_CAPS)
    if any(c <= 0 or c > 256 for c in caps):
        raise ValueError(f"DISTLEARN_CHANNEL_CAPS: caps must be in 1..256, got {caps}")
    return sorted(set(caps))


def agree_channel_caps(comm, caps: List[int]) -> List[int]:
    """Check that every rank measures the same channel-cap list.
    Each rank derives it from its own environment; a rank whose list differs
    would rebuild its communicator at another cap and the ranks would hang in
    comm init or the policy broadcast.  Collective over the control plane:
    raises ``ValueError`` naming the disagreement instead."""
    if getattr(comm, "world_size", 1) <= 1:
        return caps
    n = 17  # count + up to 16 caps
    if len(caps) > n - 1:
        raise ValueError(f"at most {n - 1} channel caps, got {caps}")
    mine = torch.zeros(n, dtype=torch.float64)
    mine[0] = len(caps)
    mine[1:1 + len(caps)] = torch.tensor([float(c) for c in caps], dtype=torch.float64)
    hi, lo = mine.clone(), -mine
    comm.all_reduce_host(hi, "max")
    comm.all_reduce_host(lo, "max")
    if not torch.equal(hi, -lo):
        raise ValueError(
            f"ranks disagree on the channel caps to measure (rank {comm.rank}: {caps}); set the same "
            "NCCL_MAX_NCHANNELS / DISTLEARN_CHANNEL_CAP / DISTLEARN_CHANNEL_CAPS on every rank")
    return caps


def runs_collectives(comm) -> bool:
    """Whether data-plane collectives on ``comm`` actually run: world > 1, or
    an RCCL communicator at world 1 with the collectives forced through RCCL
    (``DISTLEARN_RCCL_WORLD1=1``: the multi-node step configuration rehearsed
    on one GPU)."""
    return getattr(comm, "world_size", 1) > 1 or getattr(comm, "_skip1", True) is False


class RcclCommunicator(Communicator):
    """Native RCCL data plane (C++), gloo control plane."""

    def __init__(self, rank: int, world_size: int, device: torch.device, ctrl_group=None,
                 timeout_s: Optional[float] = None):
        self.ctrl = ctrl_group
        self.rank, self.world_size = rank, world_size
        self.device = torch.device(device)
        # world 1 collectives are the identity and skipped; DISTLEARN_RCCL_WORLD1=1
        # issues them anyway (exercises RCCL inside hipGraph capture on one GPU)
        self._skip1 = world_size == 1 and os.environ.get("DISTLEARN_RCCL_WORLD1", "0") != "1"
        # watchdog (csrc/comm/communicator.h): a collective older than timeout_s,
        # or an RCCL async error, aborts the communicator instead of hanging
        self.timeout_s = comm_timeout() if timeout_s is None else float(timeout_s)
        self._in_group = 0
        self._c = None
        # channel cap (maxCTAs) of this communicator; 0 = RCCL's own choice (nothing runs)
        self.channel_cap = 0
        self._init_native(rccl_channel_cap() if runs_collectives(self) else 0)

    def _init_native(self, cap: int) -> None:
        """(Re)create the native communicator with ``cap`` channels at most
        (collective: every rank calls it with the same cap)."""
        C = native()
        uid = C.rccl_unique_id() if self.rank == 0 else None
        if self.world_size > 1:
            lst = [uid]
            dist.broadcast_object_list(lst, src=0, group=self.ctrl)
            uid = lst[0]
        if self._c is not None:
            self._c.destroy()
        self._c = C.RcclCommunicator(uid, self.rank, self.world_size, self.device.index or 0, self.timeout_s,
                                     int(cap))
        self.channel_cap = int(cap)
        # CUs a concurrent collective's workgroups hold (executor CU-reserve policy)
        self.cu_reserve = int(cap)

    def set_channel_cap(self, cap: int) -> None:
        """Rebuild the communicator with another channel cap (collective).  No
        hipGraph holding collectives of the old communicator may remain."""
        if int(cap) != self.channel_cap:
            torch.cuda.synchronize(self.device)
            self._init_native(int(cap))

    @staticmethod
    def _check(t):
        if not t.is_cuda:
            raise ValueError("RcclCommunicator: GPU tensors only (use the gloo communicator for CPU)")
        if not t.is_contiguous():
            raise ValueError("RcclCommunicator: tensor must be contiguous")

    def all_reduce(self, t, op="sum", stream=None):
        self._check(t)
        self._note("all_reduce", t, OP_CODES[op])
        if self._skip1:  # identity (in place); skips RCCL's self-copy
            return
        self._call(self._c.all_reduce, t.data_ptr(), t.data_ptr(), t.numel(), DTYPE_CODES[t.dtype], OP_CODES[op],
                           stream_handle(stream))

    def broadcast(self, t, root=0, stream=None):
        self._check(t)
        self._note("broadcast", t, root)
        if self._skip1:
            return
        self._call(self._c.broadcast, t.data_ptr(), t.data_ptr(), t.numel(), DTYPE_CODES[t.dtype], root, stream_handle(stream))

    def all_gather(self, out, t, stream=None):
        self._check(t)
        self._check(out)
        self._note("all_gather", t)
        self._call(self._c.all_gather, t.data_ptr(), out.data_ptr(), t.numel(), DTYPE_CODES[t.dtype], stream_handle(stream))

    def reduce_scatter(self, out, t, op="sum", stream=None):
        self._check(t)
        self._note("reduce_scatter", t, OP_CODES[op])
        self._call(self._c.reduce_scatter, t.data_ptr(), out.data_ptr(), out.numel(), DTYPE_CODES[t.dtype], OP_CODES[op],
                               stream_handle(stream))

    def send(self, t, peer, stream=None):
        self._check(t)
        self._call(self._c.send, t.data_ptr(), t.numel(), DTYPE_CODES[t.dtype], peer, stream_handle(stream))

    def recv(self, t, peer, stream=None):
        self._check(t)
        self._call(self._c.recv, t.data_ptr(), t.numel(), DTYPE_CODES[t.dtype], peer, stream_handle(stream))

    @contextlib.contextmanager
    def group(self):
        self._c.group_start()
        try:
            yield
        finally:
            self._c.group_end()

    def health(self) -> str:
        return "communicator closed" if self._c is None else self._c.async_error()

    def pause_watch(self, paused: bool) -> None:
        """Suspend (True) / resume the watchdog's event and async-error polling
        -- around a hipGraph capture, where a HIP query from the watchdog
        thread can invalidate the capture (engine.py _capturing)."""
        if getattr(self, "_c", None) is not None:
            self._c.set_paused(bool(paused))

    def track(self, stream=None) -> None:
        """Hand the work enqueued so far on ``stream`` to the watchdog (used
        after replaying a hipGraph that contains captured collectives)."""
        if self.world_size > 1 or not self._skip1:
            self._call(self._c.track, stream_handle(stream))

    def set_timeout(self, seconds: float) -> None:
        self.timeout_s = float(seconds)
        self._c.set_timeout(self.timeout_s)

    def _call(self, fn, *args):
        try:
            return fn(*args)
        except RuntimeError as e:
            if "RCCL communicator failed" in str(e):
                raise CommError(str(e)) from e
            raise

    def close(self):
        if getattr(self, "_c", None) is not None:
            self._c.destroy()
            self._c = None


# ---------------------------------------------------------------------------
# bootstrap
# ---------------------------------------------------------------------------
def _env_int(name, default):
    v = os.environ.get(name)
    return int(v) if v not in (None, "") else default


def init_communicator(rank: Optional[int] = None, world_size: Optional[int] = None, host: Optional[str] = None,
                      port: Optional[int] = None, device=None, backend: str = "auto",
                      timeout_s: Optional[float] = None) -> Communicator:
    """Rendezvous + communicator construction.

    ``rank``/``world_size`` default to the torchrun env (RANK/WORLD_SIZE).
    ``host``/``port`` default to MASTER_ADDR/MASTER_PORT (127.0.0.1:29500).
    ``backend``: ``auto`` (RCCL for CUDA devices, gloo otherwise), ``rccl``,
    ``nccl`` (torch's process group) or ``gloo``.  ``timeout_s`` (default
    :func:`comm_timeout`) bounds every control-plane operation and arms the
    RCCL watchdog.
    """
    timeout_s = comm_timeout() if timeout_s is None else float(timeout_s)
    rank = _env_int("RANK", 0) if rank is None else rank
    world_size = _env_int("WORLD_SIZE", 1) if world_size is None else world_size
    host = host or os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = port or _env_int("MASTER_PORT", 29500)
    dev = torch.device(device) if device is not None else torch.device("cpu")
    if not dist.is_initialized():
        if world_size == 1:
            # one process: an in-memory store, no TCP listener (a port another
            # process grabbed between the launcher's probe and this bind used to
            # fail a single-node run with EADDRINUSE)
            dist.init_process_group("gloo", store=dist.HashStore(), rank=0, world_size=1,
                                    timeout=datetime.timedelta(seconds=timeout_s))
        else:
            dist.init_process_group("gloo", init_method=f"tcp://{host}:{port}", rank=rank, world_size=world_size,
                                    timeout=datetime.timedelta(seconds=timeout_s))
    ctrl = dist.group.WORLD
    if backend == "auto":
        backend = "rccl" if dev.type == "cuda" else "gloo"
    if backend == "rccl":
        return RcclCommunicator(rank, world_size, dev, ctrl_group=ctrl, timeout_s=timeout_s)
    if backend == "nccl":
        comm = ProcessGroupCommunicator(dist.new_group(backend="nccl"), ctrl)
    elif backend == "gloo":
        comm = ProcessGroupCommunicator(ctrl, ctrl)
    else:
        raise ValueError(f"unknown backend {backend!r}")
    comm.timeout_s = timeout_s
    return comm
