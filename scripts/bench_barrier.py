"""Price of s_barrier rounds in conv-kernel-shaped launches (testing/diag.hip
barrier_loop): us per round for 256/512-thread workgroups at one per CU."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native

T = _native.testing()
s = torch.cuda.current_stream().cuda_stream
sink = torch.zeros(4096, device="cuda")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for threads in (256, 512):
    for mode in (0, 1, 2):
        for n in (0, 2000):
            T.barrier_loop(256, threads, n, mode, 128 * 1024, sink.data_ptr(), s)
        torch.cuda.synchronize()
        res = []
        for n in (0, 2000):
            e0.record()
            T.barrier_loop(256, threads, n, mode, 128 * 1024, sink.data_ptr(), s)
            e1.record()
            torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3)
        print(f"threads {threads} mode {mode}: {(res[1] - res[0]) / 2000 * 1e3:.1f} ns per round "
              f"(launch {res[0]:.1f} us)", flush=True)
