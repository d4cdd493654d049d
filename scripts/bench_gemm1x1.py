#!/usr/bin/env python3
"""ResNet-50 1x1 convolutions (batch 256) on the hand-written MFMA kernels vs
MIOpen (torch conv2d, channels-last bf16): forward / dgrad / wgrad time,
achieved TFLOP/s and HBM GB/s (minimum bytes: read operands + write result).
One JSON line per shape."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3  # us


def main():
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.ops.conv import _plan_1x1 as _fwd_plan, _wgrad_plan

    C = _native.native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    shapes = [(56, 64, 64), (56, 64, 256), (56, 256, 64), (28, 512, 128), (28, 128, 512), (14, 1024, 256),
              (14, 256, 1024), (7, 2048, 512), (7, 512, 2048)]
    N = int(os.environ.get("BATCH", "256"))
    for hw, cin, cout in shapes:
        M = N * hw * hw
        x = torch.randn(N, cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, device=dev) * 0.05).to(torch.bfloat16)
        wt = w.t().contiguous()
        dy = torch.randn(N, cout, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        y = torch.empty_like(dy)
        dx = torch.empty_like(x)
        gw = torch.zeros(cout, cin, device=dev)
        rows = torch.empty(4 * max(1, (M + 127) // 128), 2, cout, device=dev)  # 4x: per-wave-row rows (bit 21)
        ft, fs = _fwd_plan(M, cout, cin)
        dt, ds = _fwd_plan(M, cin, cout)
        wtile, wsp = _wgrad_plan(cout, cin, M)
        slab = torch.empty(max(fs, ds, 1) * M * max(cin, cout), device=dev) if max(fs, ds) > 1 else torch.empty(1, device=dev)
        wslab = torch.empty(wsp * cout * cin, device=dev)
        t = {
            "fwd": timeit(lambda: C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0, slab.data_ptr(), M, 1, 1, cin,
                                             cout, 1, ft, fs, s)),
            "fwd_stats": timeit(lambda: C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), rows.data_ptr(),
                                                   slab.data_ptr(), M, 1, 1, cin, cout, 1, ft, fs, s)),
            "dgrad": timeit(lambda: C.conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, slab.data_ptr(), M, 1, 1,
                                               cout, cin, 1, dt, ds, s)),
            "wgrad": timeit(lambda: (C.conv_wgrad(dy.data_ptr(), x.data_ptr(), wslab.data_ptr(), M, 1, 1, cin, cout, 1,
                                                  wsp, cin, wtile, 0, s),
                                     C.slab_reduce_add(wslab.data_ptr(), gw.data_ptr(), wsp, cout, 1, cin, cin, s))),
        }
        w4 = w.view(cout, cin, 1, 1)
        t["miopen_fwd"] = timeit(lambda: F.conv2d(x, w4))
        t["miopen_dgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w4, None, (1, 1), (0, 0), (1, 1),
                                                                                False, (0, 0), 1, (True, False, False)))
        t["miopen_wgrad"] = timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w4, None, (1, 1), (0, 0), (1, 1),
                                                                                False, (0, 0), 1, (False, True, False)))
        if os.environ.get("SWEEP"):
            for st, wv in ((2, 8), (3, 8), (4, 8), (2, 4), (3, 4)):
                C.set_conv_stages(st, 0)
                C.set_conv_waves(wv)
                for tl in (0, 2, 1):
                    if cout % (128 if tl == 0 else 64) == 0:
                        t[f"fwd_st{st}_w{wv}_t{tl}"] = timeit(lambda: C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), 0,
                                                                         slab.data_ptr(), M, 1, 1, cin, cout, 1, tl, 1, s))
                    if cin % (128 if tl == 0 else 64) == 0:
                        t[f"dgrad_st{st}_w{wv}_t{tl}"] = timeit(lambda: C.conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0,
                                                                           slab.data_ptr(), M, 1, 1, cout, cin, 1, tl, 1, s))
            C.set_conv_stages(3, 0)
            C.set_conv_waves(8)
            C.set_conv_stages(3, 0)
            for tl in (1, 2):
                if cout % (64 if tl == 1 else 128):
                    continue
                for sp in sorted({max(2, wsp // d) for d in (4, 2, 1)} | {wsp * 2}):
                    ws = torch.empty(sp * cout * cin, device=dev)
                    t[f"wgslab_t{tl}_s{sp}"] = timeit(lambda: (C.conv_wgrad(
                        dy.data_ptr(), x.data_ptr(), ws.data_ptr(), M, 1, 1, cin, cout, 1, sp, cin, tl, 0, s),
                        C.slab_reduce(ws.data_ptr(), gw.data_ptr(), sp, cout, 1, cin, cin, s)))
        flops = 2.0 * M * cin * cout
        by = {"fwd": 2 * M * (cin + cout), "dgrad": 2 * M * (cin + cout), "wgrad": 2 * M * (cin + cout)}
        out = {"hw": hw, "cin": cin, "cout": cout, "M": M, "plans": [ft, fs, dt, ds, wtile, wsp]}
        for k, v in t.items():
            base = k.replace("miopen_", "").replace("_stats", "").replace("wgslab", "wgrad").split("_")[0]
            out[k] = {"us": round(v, 1), "TFLOPs": round(flops / v / 1e6, 1), "GBs": round(by[base] / v / 1e3, 0)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
