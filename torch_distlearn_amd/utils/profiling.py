"""Step / communication timing (the reference has no tracing).

* :class:`StepTimer` -- wall-clock per step with device synchronisation,
  images/s.
* :class:`CommTimer` -- HIP events recorded on the comm stream around every
  bucket all-reduce (no host synchronisation on the hot path); ``summary()``
  reports total communication time and how much of it overlapped compute
  (events on the compute stream bracket the backward).
* :func:`torch_profile` -- a ``torch.profiler`` context that exports a Chrome
  trace; for per-kernel counters use ``rocprofv3 --kernel-trace --stats``
  (scripts/prof_summary.py summarises its database).
"""
from __future__ import annotations

import contextlib
import time
from typing import List, Optional

import torch


class StepTimer:
    def __init__(self, sync: bool = True):
        self.sync = sync and torch.cuda.is_available()
        self.times: List[float] = []
        self._t = None

    def start(self):
        if self.sync:
            torch.cuda.synchronize()
        self._t = time.perf_counter()

    def stop(self, items: int = 0) -> float:
        if self.sync:
            torch.cuda.synchronize()
        dt = time.perf_counter() - self._t
        self.times.append(dt)
        self.items = items
        return dt

    def rate(self, items_per_step: int) -> float:
        return items_per_step * len(self.times) / max(sum(self.times), 1e-12)


class CommTimer:
    """Attach to a GradBucketer: ``CommTimer(bucketer)``; call ``begin_step()``
    before forward and ``end_step()`` after the optimizer step."""

    def __init__(self, bucketer):
        self.b = bucketer
        self.enabled = bucketer is not None and bucketer.cuda
        self.records = []
        self._cur = None
        if self.enabled:
            orig = bucketer._launch

            def timed_launch(i, _orig=orig):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record(self.b.stream)
                _orig(i)
                e.record(self.b.stream)
                if self._cur is not None:
                    self._cur["buckets"].append((s, e))

            bucketer._launch = timed_launch

    def begin_step(self):
        if not self.enabled:
            return
        s = torch.cuda.Event(enable_timing=True)
        s.record()
        self._cur = {"start": s, "buckets": []}

    def end_step(self):
        if not self.enabled or self._cur is None:
            return
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        self._cur["end"] = e
        self.records.append(self._cur)
        self._cur = None

    def summary(self) -> dict:
        if not self.records:
            return {}
        torch.cuda.synchronize()
        step_ms = comm_ms = exposed_ms = 0.0
        for r in self.records:
            step_ms += r["start"].elapsed_time(r["end"])
            for s, e in r["buckets"]:
                comm_ms += s.elapsed_time(e)
            if r["buckets"]:
                # communication still running after the last compute event is exposed
                last = r["buckets"][-1][1]
                exposed_ms += max(0.0, r["end"].elapsed_time(last))
        n = len(self.records)
        return {"steps": n, "step_ms": step_ms / n, "comm_ms": comm_ms / n, "exposed_comm_ms": exposed_ms / n,
                "overlap_fraction": 1.0 - (exposed_ms / comm_ms if comm_ms > 0 else 0.0)}


@contextlib.contextmanager
def torch_profile(trace_path: Optional[str] = None):
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        yield prof
    if trace_path:
        prof.export_chrome_trace(trace_path)
