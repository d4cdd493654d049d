"""Step / communication timing (the reference has no tracing).

* :class:`StepTimer` -- wall-clock per step with device synchronisation,
  images/s.
* :func:`comm_summary` -- communication time / exposed time / overlap
  fraction from the events the gradient bucketer records while profiling
  (``DataParallelTrainer.comm_profile``: eager calibration steps outside any
  captured hipGraph, training state restored afterwards).
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


def comm_summary(records, world_size: int = 1) -> dict:
    """Summarise :class:`~torch_distlearn_amd.parallel.buckets.GradBucketer`
    profile records (HIP events on the comm stream around every bucket
    all-reduce, and on the compute stream where the backward ends and where
    the update may start):

    * ``comm_ms``          -- summed all-reduce time per step (comm stream busy);
    * ``exposed_comm_ms``  -- time the compute stream waits for communication
      after its backward is done (the part NOT hidden behind backward);
    * ``overlap_fraction`` -- 1 - exposed / comm, clamped to [0, 1] (the
      exposed wait also holds the event / queue latency of the last bucket);
    * ``busbw_GBps``       -- ring bus bandwidth of the bucket all-reduces,
      2 (n-1)/n * bytes / comm time, with n = ``world_size`` (0 at world 1).
    """
    recs = [r for r in records if r.get("buckets") and "comm_joined" in r]
    if not recs:
        return {}
    torch.cuda.synchronize()
    comm = exposed = 0.0
    nbytes = 0
    for r in recs:
        comm += sum(s.elapsed_time(e) for s, e, _ in r["buckets"])
        nbytes += sum(b for _, _, b in r["buckets"])
        exposed += max(0.0, r["compute_done"].elapsed_time(r["comm_joined"]))
    n = len(recs)
    return {"steps": n, "comm_ms": round(comm / n, 4), "exposed_comm_ms": round(exposed / n, 4),
            # exposed can exceed comm when issue latency dominates tiny collectives: clamp
            "overlap_fraction": round(min(1.0, max(0.0, 1.0 - (exposed / comm if comm > 0 else 0.0))), 4),
            "bytes_per_step": nbytes // n, "buckets": len(recs[0]["buckets"]),
            "busbw_GBps": round(2.0 * (world_size - 1) / world_size * (nbytes / n) / (comm / n * 1e6), 2)
            if comm > 0 and world_size > 1 else 0.0}


@contextlib.contextmanager
def torch_profile(trace_path: Optional[str] = None):
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts) as prof:
        yield prof
    if trace_path:
        prof.export_chrome_trace(trace_path)
