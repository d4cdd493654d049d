"""Bucketed gradient all-reduce overlapped with backward.

The reference starts communication only after the whole backward finished and
then ships 18 tensors one by one through a TCP tree (SURVEY §3.2 "No
overlap").  On MI355X the flat gradient buffer of a :class:`FlatParams` is cut
into contiguous buckets in reverse registration order (backward produces the
last layers first).  As soon as every gradient of a bucket has been
accumulated, the bucket's RCCL all-reduce is issued on a high-priority comm
stream (event-ordered after the producing kernels), so it runs over xGMI while
the earlier layers' backward is still computing.  Buckets are always launched
in index order, so every node issues the identical collective sequence
(required by RCCL).

Bucket sizing for 7 xGMI links per GPU: a ring all-reduce splits a
bucket into world x channels chunks; keeping chunks >= ~64-128 KB needs buckets
of a few MB.  Default 4 MiB.

The participation slot (``n``) lives in the header of the flat buffer, which
is inside the bucket launched *last*, so ``n`` is complete once all buckets
have landed; draining nodes replay the same bucket sequence with zeros and
slot 0 (:meth:`drain`).

Wire dtype (``wire="bf16"``): each bucket's fp32 gradient is
cast to the FlatParams' bf16 wire buffer on the comm stream and THAT copy is
all-reduced -- half the xGMI bytes per step -- while the header (participation
count) is all-reduced in fp32 beside it in the same group.  The fused SGD
reads the bf16 result directly (``AllReduceSGD.step``); API callers that read
``flat.grad`` get it widened back to fp32 by :meth:`finish`.  At world 1 the
all-reduce is the identity and the wire stays fp32.  Accuracy trade-off: the
collective reduces in its wire dtype, so the gradient SUM is accumulated in
bf16 at every ring hop -- on top of rounding each rank's gradient to bf16 the
sum picks up about one bf16 rounding per hop, i.e. its relative error grows
with the world size (measured bound: tests/distributed/test_allreduce_sgd.py
test_bf16_wire_matches_fp32_wire, worlds 2-8).  Replicas stay bitwise
identical (every rank applies the same reduced bytes).  The headline bench
keeps the fp32 wire.

Per-bucket update (:meth:`set_early_update`, used by the native executors):
the fused SGD of a bucket's parameters runs on the comm stream right after
that bucket's all-reduce, so the update of the largest (last-layer) bucket
overlaps the earlier layers' backward instead of one full-buffer SGD kernel
after the last bucket lands.  The participation count is then all-reduced
with the FIRST launched bucket (in the same group, fp32), so every bucket's
update already divides by the final ``n``; draining nodes issue the same
collectives and apply no update.  Only valid when nothing reads a bucket's
parameters after its gradients are final (true for the HIP executors: the
dgrads read the step's transposed weight copies).
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

import contextlib

from ..ops.flat import HEADER, SLOT, FlatParams, cast_, fill_


def _nullctx():
    return contextlib.nullcontext()


class _Stamp:
    """A device timestamp (native ``stamp_time``: the constant-rate wall clock)
    with the ``elapsed_time`` interface of a HIP event, read after the work that
    wrote it has finished."""

    _khz = None

    def __init__(self, buf, i):
        self.buf, self.i = buf, i

    @classmethod
    def record(cls, stamps, stream):
        from .._native import native

        buf, i = stamps
        if i >= buf.numel():
            raise RuntimeError("capture profile: out of timestamp slots")
        stamps[1] = i + 1
        native().stamp_time(buf.data_ptr() + 8 * i, stream.cuda_stream)
        return cls(buf, i)

    def elapsed_time(self, end) -> float:
        if _Stamp._khz is None:
            from .._native import native

            _Stamp._khz = native().wall_clock_khz()
        return float(int(end.buf[end.i]) - int(self.buf[self.i])) / _Stamp._khz  # ms


class GradBucketer:
    def __init__(self, comm, flat: FlatParams, bucket_bytes: int = 4 << 20, hooks: bool = True,
                 stream: Optional["torch.cuda.Stream"] = None, wire: str = "fp32"):
        if wire not in ("fp32", "bf16"):
            raise ValueError(f"wire dtype {wire!r}: fp32 or bf16")
        self.comm = comm
        self.flat = flat
        # bf16 wire only where a collective actually runs (world 1 skips it unless forced)
        self.wire16 = wire == "bf16" and (comm.world_size > 1 or getattr(comm, "_skip1", True) is False)
        self.wire = "bf16" if self.wire16 else "fp32"
        if self.wire16:
            flat.enable_grad16()
        self.ranges: List[Tuple[int, int]] = flat.buckets(bucket_bytes)
        self.nb = len(self.ranges)
        # leaf -> bucket
        self.leaf_bucket = []
        for off in flat.offsets:
            for b, (s, e) in enumerate(self.ranges):
                if s <= off < e:
                    self.leaf_bucket.append(b)
                    break
        self.need = [0] * self.nb
        for b in self.leaf_bucket:
            self.need[b] += 1
        self.cuda = flat.data.is_cuda
        # communication profile (utils/profiling.py): a list while enabled; eager
        # steps, or -- profile_in_capture -- a hipGraph capture, whose event-record
        # nodes re-record the same events at every replay
        # (DataParallelTrainer.comm_profile(replay=True))
        self.profile = None
        self.profile_in_capture = False
        self._rec = None
        self.stream = stream if stream is not None else (
            torch.cuda.Stream(device=flat.device, priority=-1) if self.cuda else None)
        # per-bucket update (set_early_update): fn(start, end, grad_buffer) on the comm stream
        self.early = None
        self.hdr_first = False  # the count rides the first launched bucket
        self._draining = False
        self.early_applied = False  # the last finish() ran every bucket's update
        self._reset()
        self._hooks = []
        if hooks:
            for i, t in enumerate(flat.leaves):
                if t.requires_grad and hasattr(t, "register_post_accumulate_grad_hook"):
                    self._hooks.append(t.register_post_accumulate_grad_hook(self._make_hook(i)))

    def _make_hook(self, i):
        def hook(_p):
            self.mark_leaf_ready(i)
        return hook

    def _reset(self):
        self.remaining = list(self.need)
        self.next = 0
        self.launched = 0

    # ---------------------------------------------------------------- launch
    def _profiling(self) -> bool:
        return (self.profile is not None and self.cuda
                and (self.profile_in_capture or not torch.cuda.is_current_stream_capturing()))

    def _event(self, stream):
        if self.profile_in_capture:
            # inside a capture: a device-timestamp kernel node (re-run at every
            # replay); a plain event record would become a fork/join edge, and HIP
            # refuses external event-record nodes (scripts/probe_graph_events.py)
            return _Stamp.record(self._stamps, stream)
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(stream)
        return ev

    def start_capture_profile(self, slots: int = 512) -> None:
        """Profile the next capture with device timestamps (``profile`` := [])."""
        self.profile, self.profile_in_capture = [], True
        self._stamps = [torch.zeros(slots, dtype=torch.int64, device=self.flat.grad.device), 0]

    def stop_capture_profile(self) -> list:
        recs, self.profile, self.profile_in_capture = self.profile, None, False
        return recs

    def set_early_update(self, fn) -> None:
        """``fn(start, end, grad)`` updates parameters [start, end) from the
        all-reduced ``grad`` buffer (fp32 grad or the bf16 wire copy) on the
        current (comm) stream; None restores the single update after finish()."""
        self.early = fn
        self.hdr_first = fn is not None and self.nb > 1

    def _reduce(self, s: int, e: int, stream=None, b: int = -1):
        """All-reduce grad[s:e] (fp32 wire) or its bf16 copy, and the fp32
        header (participation count) exactly once per step: with the bucket
        that holds it, or -- per-bucket updates -- with the first bucket."""
        f = self.flat
        hdr_here = (b == 0) if self.hdr_first else (s < HEADER)
        if self.hdr_first and s < HEADER:
            s = HEADER  # the header went with bucket 0
        if not self.wire16:
            if hdr_here and s >= HEADER:
                with self.comm.group():
                    self.comm.all_reduce(f.grad[s:e], "sum", stream=stream)
                    self.comm.all_reduce(f.grad[0:HEADER], "sum", stream=stream)
            else:
                self.comm.all_reduce(f.grad[s:e], "sum", stream=stream)
            return
        s16 = max(s, HEADER)  # the bf16 copy of the header is never read
        cast_(f.grad16[s16:e], f.grad[s16:e])
        with self.comm.group():
            self.comm.all_reduce(f.grad16[s16:e], "sum", stream=stream)
            if hdr_here:  # the participation count stays exact in fp32
                self.comm.all_reduce(f.grad[0:HEADER], "sum", stream=stream)

    def _launch(self, b: int):
        s, e = self.ranges[b]
        buf = (self.flat.grad16 if self.wire16 else self.flat.grad)[s:e]
        if self.cuda:
            cur = torch.cuda.current_stream()
            self.stream.wait_stream(cur)
            prof = self._profiling()
            if prof:
                if self._rec is None:
                    self._rec = {"buckets": []}
                t0 = self._event(self.stream)
            with torch.cuda.stream(self.stream):
                self._reduce(s, e, stream=self.stream, b=b)
                if self.early is not None and not self._draining:
                    self.early(max(s, HEADER), e, self.flat.grad16 if self.wire16 else self.flat.grad)
            if prof:
                self._rec["buckets"].append((t0, self._event(self.stream), (e - s) * buf.element_size()))
            buf.record_stream(self.stream)
        else:
            self._reduce(s, e, b=b)
            if self.early is not None and not self._draining:
                self.early(max(s, HEADER), e, self.flat.grad16 if self.wire16 else self.flat.grad)
        self.launched += 1

    def _pump(self):
        while self.next < self.nb and self.remaining[self.next] <= 0:
            self._launch(self.next)
            self.next += 1

    def mark_leaf_ready(self, i: int):
        b = self.leaf_bucket[i]
        self.remaining[b] -= 1
        self._pump()

    def mark_bucket_ready(self, b: int):
        """Explicit-executor path: every gradient of bucket ``b`` is written."""
        self.remaining[b] = 0
        self._pump()

    def finish(self, widen: bool = True):
        """Launch what is left (params without grads), then order the compute
        stream after the comm stream.  Resets for the next step.  With the
        bf16 wire, ``widen`` copies the all-reduced bf16 gradient back into
        ``flat.grad`` (callers that read the bf16 copy pass False)."""
        for b in range(self.nb):
            self.remaining[b] = 0
        self._pump()
        self.early_applied = self.early is not None and not self._draining
        if self.wire16 and widen:
            f = self.flat
            ctx = torch.cuda.stream(self.stream) if self.cuda else _nullctx()
            with ctx:
                cast_(f.grad[HEADER:], f.grad16[HEADER:])
        if self.cuda:
            cur = torch.cuda.current_stream()
            prof = self._profiling() and self._rec is not None
            if prof:
                self._rec["compute_done"] = self._event(cur)   # backward finished on the compute stream
            cur.wait_stream(self.stream)
            if prof:
                self._rec["comm_joined"] = self._event(cur)    # the update may start
                self.profile.append(self._rec)
        self._rec = None
        self._reset()

    def drain(self):
        """Replay zero buckets (slot 0) until no node is active any more."""
        self._draining = True  # same collectives, no parameter update
        try:
            while True:
                fill_(self.flat.grad, 0.0, slot_value=0.0)
                self.finish(widen=False)
                n = int(self.flat.grad[SLOT].item())
                if n == 0:
                    return
        finally:
            self._draining = False

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
