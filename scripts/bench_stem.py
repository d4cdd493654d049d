#!/usr/bin/env python3
"""ResNet-50 stem forward (7x7/2 conv, 3 -> 64, batch 256) on the MFMA
kernels: the 2x2 space-to-depth form (4x4 stride-1 conv over 16 channels,
ops/conv.py StemConv) per tile / wave config, against the same GEMM with the
four horizontal taps folded into the channels (4x1 conv over 64 channels,
S4[n][i][j][kw*16 + c] = S[n][i][j + kw][c]).  One JSON line."""
import json
import os
import sys

import torch

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
    return s.elapsed_time(e) / n * 1e3


def main():
    from torch_distlearn_amd import _native

    C = _native.native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    N, H, cout = int(os.environ.get("BATCH", "256")), 224, 64
    Ho = Wo = 112
    Hs = Ws = Ho + 3
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(N, 3, H, H, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    S = torch.empty(N, Hs, Ws, 16, dtype=torch.bfloat16, device=dev)
    C.s2d_stem_input(x.data_ptr(), S.data_ptr(), N, H, H, Hs, Ws, 3, s)
    w4 = (torch.randn(cout, 4, 4, 16, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    y = torch.empty(N, Ho, Wo, cout, dtype=torch.bfloat16, device=dev)
    out = {"s2d_input_us": round(timeit(lambda: C.s2d_stem_input(x.data_ptr(), S.data_ptr(), N, H, H, Hs, Ws, 3, s)), 1)}
    for name, tile in (("t2_w8", 2 | (3 << 4) | (8 << 8)), ("t2", 2), ("t2_w4", 2 | (3 << 4) | (4 << 8)),
                       ("t1", 1), ("t2_again", 2), ("t2_w8_again", 2 | (3 << 4) | (8 << 8)),
                       ("t2_sw", 2 | (1 << 21)), ("t2_w8_sw", 2 | (3 << 4) | (8 << 8) | (1 << 21))):
        out["s2d16_" + name] = round(timeit(lambda: C.conv_fwd_ex(S.data_ptr(), w4.data_ptr(), y.data_ptr(), 0, 0, N, Ho,
                                                                   Wo, Hs, Ws, 16, cout, 4, 4, 1, 0, 0, 0, 0, 0, 0,
                                                                   tile, 1, s)), 1)
    ref = y.clone()
    S4 = torch.stack([S[:, :, kw:kw + Wo, :] for kw in range(4)], dim=3).reshape(N, Hs, Wo, 64).contiguous()
    for name, tile in (("t2", 2), ("t2_st2_w4", 2 | (2 << 4) | (4 << 8)), ("t2_st2_w8", 2 | (2 << 4) | (8 << 8)),
                       ("t2_st3_w4", 2 | (3 << 4) | (4 << 8)), ("t2_st3_w8", 2 | (3 << 4) | (8 << 8)), ("t1", 1)):
        out["fold64_" + name] = round(timeit(lambda: C.conv_fwd_ex(S4.data_ptr(), w4.data_ptr(), y.data_ptr(), 0, 0, N,
                                                                    Ho, Wo, Hs, Wo, 64, cout, 4, 1, 1, 0, 0, 0, 0, 0,
                                                                    0, tile, 1, s)), 1)
    out["fold64_max_abs_diff"] = float((y.float() - ref.float()).abs().max())
    out["fold64_copy_us"] = round(timeit(lambda: torch.stack([S[:, :, kw:kw + Wo, :] for kw in range(4)], dim=3)), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
