"""Probe: do HIP event-record nodes (hipEventRecordWithFlags(..., External))
inside a captured graph time the replay?  One case per process (a failed
capture can leave a sticky error).  python scripts/probe_graph_events.py [case]"""
import subprocess
import sys
import traceback

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def case(kind):
    from torch_distlearn_amd._native import native
    C = native()
    x = torch.zeros(1 << 22, device="cuda")
    s = torch.cuda.Stream()
    side = torch.cuda.Stream()
    e0, e1 = C.TimingEvent(), C.TimingEvent()
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        x.add_(1)  # warm-up
    torch.cuda.synchronize()
    stage = "capture"
    try:
        with torch.cuda.graph(g, stream=s, capture_error_mode="thread_local"):
            cur = torch.cuda.current_stream()
            if kind == "same":
                e0.record(cur.cuda_stream, True)
                for _ in range(20):
                    x.add_(1)
                e1.record(cur.cuda_stream, True)
            else:  # fork onto a side stream, events there, join back
                side.wait_stream(cur)
                with torch.cuda.stream(side):
                    e0.record(side.cuda_stream, True)
                    for _ in range(20):
                        x.add_(1)
                    e1.record(side.cuda_stream, True)
                cur.wait_stream(side)
        stage = "replay"
        for i in range(3):
            g.replay()
            torch.cuda.synchronize()
            stage = "elapsed"
            print(kind, "replay", i, "ms", e0.elapsed_time(e1), "x", float(x[0]), flush=True)
        print(kind, "OK")
    except Exception:
        print(kind, "FAILED at", stage)
        traceback.print_exc()


if __name__ == "__main__":
    if len(sys.argv) > 1:
        case(sys.argv[1])
    else:
        for k in ("same", "fork"):
            r = subprocess.run([sys.executable, __file__, k], timeout=120)
            print("case", k, "rc", r.returncode, flush=True)
