#!/usr/bin/env python3
"""Would hand-written 3x3 convolutions pay for ResNet-50?  MIOpen (torch,
channels-last bf16, solver search on) forward / dgrad / wgrad on the four
stride-1 3x3 bottleneck shapes at batch 256, vs the hand-written streaming
implicit-GEMM kernels (conv_fwd / conv_wgrad) on the nearest power-of-two
spatial size (they need pow2 H, W today), compared per TFLOP/s."""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
torch.backends.cudnn.benchmark = True


def timeit(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.models.cifar_hip import _fwd_plan, _wgrad_plan

    C = _native.native()
    if os.environ.get("REGION") is not None:  # 0: streaming kernel only (what non-pow2 shapes would get)
        C.set_conv_region(int(os.environ["REGION"]))
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    B = 256
    for hw, c, hw2 in [(56, 64, 64), (28, 128, 32), (14, 256, 16), (7, 512, 8)]:
        out = {"hw": hw, "c": c}
        x = torch.randn(B, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(c, c, 3, 3, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dy = torch.randn(B, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        fl = 2.0 * B * hw * hw * c * c * 9
        t = {"fwd": timeit(lambda: F.conv2d(x, w, None, 1, 1)),
             "dgrad": timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False,
                                                                         (0, 0), 1, (True, False, False))),
             "wgrad": timeit(lambda: torch.ops.aten.convolution_backward(dy, x, w, None, (1, 1), (1, 1), (1, 1), False,
                                                                         (0, 0), 1, (False, True, False)))}
        for k, v in t.items():
            out["miopen_" + k] = {"us": round(v, 1), "TFLOPs": round(fl / v / 1e6)}
        # hand-written kernels on [B, hw2, hw2, c] (zero-bordered input, KS = 3)
        M, K = B * hw2 * hw2, 9 * c
        xp = F.pad(torch.randn(B, hw2, hw2, c, device=dev), (0, 0, 1, 1, 1, 1)).to(torch.bfloat16)
        dyp = F.pad(torch.randn(B, hw2, hw2, c, device=dev), (0, 0, 1, 1, 1, 1)).to(torch.bfloat16)
        w2 = (torch.randn(c, 3, 3, c, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(B, hw2, hw2, c, dtype=torch.bfloat16, device=dev)
        fl2 = 2.0 * M * c * K
        ft, fs = _fwd_plan(M, c, K)
        slab = torch.empty(max(fs, 1) * M * c + 1, device=dev)
        wt, wsp = _wgrad_plan(c, K, M)
        wslab = torch.empty(wsp * c * K, device=dev)
        t2 = {"fwd": timeit(lambda: C.conv_fwd(xp.data_ptr(), w2.data_ptr(), y.data_ptr(), 0, slab.data_ptr(), B, hw2,
                                               hw2, c, c, 3, ft, fs, s)),
              "wgrad": timeit(lambda: C.conv_wgrad(dyp.data_ptr(), xp.data_ptr(), wslab.data_ptr(), B, hw2, hw2, c, c, 3,
                                                   wsp, K, wt, 0, s))}
        for k, v in t2.items():
            out["hip_pow2_" + k] = {"us": round(v, 1), "TFLOPs": round(fl2 / v / 1e6), "hw": hw2}
        # the actual (non-pow2) shape on the streaming kernels
        M3 = B * hw * hw
        xq = F.pad(torch.randn(B, hw, hw, c, device=dev), (0, 0, 1, 1, 1, 1)).to(torch.bfloat16)
        dyq = F.pad(torch.randn(B, hw, hw, c, device=dev), (0, 0, 1, 1, 1, 1)).to(torch.bfloat16)
        yq = torch.empty(B, hw, hw, c, dtype=torch.bfloat16, device=dev)
        ft3, fs3 = _fwd_plan(M3, c, K)
        slab3 = torch.empty(max(fs3, 1) * M3 * c + 1, device=dev)
        wt3, wsp3 = _wgrad_plan(c, K, M3)
        wslab3 = torch.empty(wsp3 * c * K, device=dev)
        t3 = {"fwd": timeit(lambda: C.conv_fwd(xq.data_ptr(), w2.data_ptr(), yq.data_ptr(), 0, slab3.data_ptr(), B, hw,
                                               hw, c, c, 3, ft3, fs3, s)),
              "wgrad": timeit(lambda: C.conv_wgrad(dyq.data_ptr(), xq.data_ptr(), wslab3.data_ptr(), B, hw, hw, c, c, 3,
                                                   wsp3, K, wt3, 0, s))}
        for k, v in t3.items():
            out["hip_actual_" + k] = {"us": round(v, 1), "TFLOPs": round(fl / v / 1e6), "plan": [ft3, fs3, wt3, wsp3]}
        if os.environ.get("SWEEP"):
            best_f, best_w = [], []
            for st, wv in ((2, 8), (3, 8), (4, 8), (2, 4), (3, 4)):
                for tl in (0, 2):
                    if c % (128 if tl == 0 else 64):
                        continue
                    for sp in (1, 2):
                        packed = tl | (st << 4) | (wv << 8)
                        sl = torch.empty(sp * M3 * c, device=dev)  # split-K slabs [sp][M][c]
                        us = timeit(lambda: C.conv_fwd(xq.data_ptr(), w2.data_ptr(), yq.data_ptr(), 0, sl.data_ptr(),
                                                       B, hw, hw, c, c, 3, packed, sp, s))
                        best_f.append((round(us, 1), f"st{st}_w{wv}_t{tl}_s{sp}"))
            for wst in (0, 3, 4):
                C.set_conv_stages(3, wst)
                for tl in (0, 1, 2):
                    if c % (64 if tl == 1 else 128):
                        continue
                    bm, bn = {2: (128, 128), 1: (64, 64), 0: (128, 64)}[tl]
                    tiles = (c // bm) * ((K + bn - 1) // bn)
                    for sp in sorted({1, 2, 4, 8, 16, 32, max(1, 256 // tiles), max(1, 512 // tiles)}):
                        if M3 // sp < 256:
                            continue
                        ws = torch.empty(sp * c * K, device=dev)
                        us = timeit(lambda: C.conv_wgrad(dyq.data_ptr(), xq.data_ptr(), ws.data_ptr(), B, hw, hw, c, c,
                                                         3, sp, K, tl, 0, s))
                        best_w.append((round(us, 1), f"wst{wst}_t{tl}_s{sp}"))
            C.set_conv_stages(3, 0)
            out["sweep_fwd"] = sorted(best_f)[:4]
            out["sweep_wgrad"] = sorted(best_w)[:4]
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
