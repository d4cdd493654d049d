"""Batch-aware conv plans: time every forward / dgrad plan
of the CIFAR layers at a given per-GPU batch -- region (tap-reuse) kernel or
streaming kernel, 128x64 / 64x64 tiles, split-K counts -- including the
split-K combine launch, and print one JSON line per (layer, plan).
    python scripts/sweep_small_batch.py --batch 4 [--iters 50] > sweep.jsonl"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native
from torch_distlearn_amd.models.cifar_hip import _fwd_plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--iters", type=int, default=40)
    a = ap.parse_args()
    C = _native.native()
    C.set_reduce_atomic(16)
    dev = torch.device("cuda")
    B = a.batch
    layers = [(16, 64, 128), (8, 128, 256), (4, 256, 512)]
    slab = torch.empty(32 * 1024 * 1024, device=dev)
    stats = torch.zeros(16 * 2 * 512, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def cur():
        return torch.cuda.current_stream().cuda_stream

    def timeit(fn):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(a.iters):
                fn()
        g.replay()
        torch.cuda.synchronize()
        ev0.record()
        g.replay()
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) * 1e3 / a.iters

    for li, (H, cin, cout) in enumerate(layers, 2):
        M = B * H * H
        x = torch.nn.functional.pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
        w = (torch.randn(cout, 5, 5, cin, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(B, H, H, cout, dtype=torch.bfloat16, device=dev)
        dy = torch.nn.functional.pad(torch.randn(B, H, H, cout, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
        wt = (torch.randn(cin, 5, 5, cout, device=dev) * 0.05).to(torch.bfloat16)
        dx = torch.empty(B, H, H, cin, dtype=torch.bfloat16, device=dev)
        for kind in ("fwd", "dgrad"):
            N, K = (cout, 25 * cin) if kind == "fwd" else (cin, 25 * cout)
            src, wgt, out = (x, w, y) if kind == "fwd" else (dy, wt, dx)
            cin_k, cout_k = (cin, cout) if kind == "fwd" else (cout, cin)
            st = stats.data_ptr() if kind == "fwd" else 0
            cur_plan = _fwd_plan(M, N, K)
            ksteps = K // 64
            for region in (1, 2, 0, -1):  # -1: streaming kernel, in-launch split-K combine (conv_fwd_fix)
                for tile in (2, 1, 0):
                    if N % (128 if tile == 0 else 64) != 0:
                        continue
                    for sp in (1, 2, 4, 8, 16, 32, 64):
                        if sp > ksteps or sp * M * N > slab.numel():
                            continue
                        if sp > 1 and 256 % (N // 8) != 0:
                            continue
                        if region == -1:
                            if not C.conv_fix_ok(B, H, H, cin_k, cout_k, 5, tile, sp):
                                continue
                        elif region and not C.conv_region_ok(B, H, H, cin_k, cout_k, 5, tile, sp):
                            continue
                        C.set_conv_region(max(region, 0))
                        try:
                            if region == -1:
                                us = timeit(lambda: C.conv_fwd_fix(src.data_ptr(), wgt.data_ptr(), out.data_ptr(), st,
                                                                   slab.data_ptr(), B, H, H, cin_k, cout_k, 5, tile,
                                                                   sp, 0, 0, 0, cur()))
                            else:
                                us = timeit(lambda: C.conv_fwd(src.data_ptr(), wgt.data_ptr(), out.data_ptr(), st,
                                                               slab.data_ptr(), B, H, H, cin_k, cout_k, 5, tile, sp,
                                                               cur()))
                        except RuntimeError as e:
                            print(json.dumps({"layer": f"{kind}{li}", "B": B, "region": region, "tile": tile,
                                              "splits": sp, "error": str(e)[:80]}), flush=True)
                            continue
                        finally:
                            C.set_conv_region(1)
                        print(json.dumps({"layer": f"{kind}{li}", "B": B, "M": M, "N": N, "K": K, "region": region,
                                          "tile": tile, "splits": sp, "us": round(us, 2),
                                          "current": [tile, sp] == list(cur_plan) and region == 1}), flush=True)


if __name__ == "__main__":
    main()
