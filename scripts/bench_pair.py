#!/usr/bin/env python3
"""Does running a CIFAR layer's wgrad and dgrad CONCURRENTLY (two streams,
eager launches) beat running them back to back?  Both are ~20 us,
latency-bound kernels with ~one workgroup per CU; this measures the headroom
a grouped (one-launch) wgrad+dgrad kernel could have.  Prints per layer:
dgrad alone, wgrad alone, sequential pair, concurrent pair (us per pair)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.models.cifar_hip import _fwd_plan, _wgrad_plan

    C = _native.native()
    C.set_conv_stages(int(os.environ.get("FWD_STAGES", "3")), 0)
    dev = torch.device("cuda")
    B, iters = 128, 200
    main_s = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    pad = torch.nn.functional.pad
    for li, (H, cin, cout) in enumerate([(16, 64, 128), (8, 128, 256), (4, 256, 512)], start=2):
        M, K = B * H * H, 25 * cin
        x = pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
        dy = pad(torch.randn(B, H, H, cout, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
        wt = torch.randn(cin, 5, 5, cout, device=dev).to(torch.bfloat16)
        dx = torch.empty(B, H, H, cin, dtype=torch.bfloat16, device=dev)
        slab_d = torch.empty(16 * 1024 * 1024, device=dev)
        slab_w = torch.empty(16 * 1024 * 1024, device=dev)
        dt, ds = _fwd_plan(M, cin, 25 * cout)
        wtile, wsp = _wgrad_plan(cout, K, M)

        def dgrad(s):
            C.conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, slab_d.data_ptr(), B, H, H, cout, cin, 5, dt,
                       ds, s.cuda_stream)

        def wgrad(s):
            C.conv_wgrad(dy.data_ptr(), x.data_ptr(), slab_w.data_ptr(), B, H, H, cin, cout, 5, wsp, K, wtile, 0,
                         s.cuda_stream)

        def timed(body):
            for _ in range(5):
                body()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for _ in range(iters):
                body()
            e1.record(main_s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / iters

        def conc():
            ev = torch.cuda.Event()
            ev.record(main_s)
            s1.wait_event(ev)
            s2.wait_event(ev)
            dgrad(s1)
            wgrad(s2)
            a, b = torch.cuda.Event(), torch.cuda.Event()
            a.record(s1)
            b.record(s2)
            main_s.wait_event(a)
            main_s.wait_event(b)

        def seq_forked():  # same fork/join event traffic, kernels serialised on s1
            ev = torch.cuda.Event()
            ev.record(main_s)
            s1.wait_event(ev)
            dgrad(s1)
            wgrad(s1)
            a = torch.cuda.Event()
            a.record(s1)
            main_s.wait_event(a)

        t_d = timed(lambda: dgrad(main_s))
        t_w = timed(lambda: wgrad(main_s))
        t_seq = timed(lambda: (dgrad(main_s), wgrad(main_s)))
        t_seqf = timed(seq_forked)
        t_con = timed(conc)
        print(f"layer{li}: dgrad {t_d:6.1f} (tile{dt} split{ds})  wgrad {t_w:6.1f} (tile{wtile} split{wsp})  "
              f"seq {t_seq:6.1f}  seq+fork {t_seqf:6.1f}  concurrent {t_con:6.1f} us", flush=True)


if __name__ == "__main__":
    main()
