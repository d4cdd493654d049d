"""Micro-benchmark of the implicit-GEMM conv kernels on the reference model's
layer shapes (per-GPU batch B): forward, dgrad, wgrad; prints us and TFLOP/s.
    python scripts/bench_conv.py [--batch 128] [--iters 50] [--only fwd2]"""

def _native_testing():
    from torch_distlearn_amd import _native

    return _native.testing()

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native
from torch_distlearn_amd.models.cifar_hip import _fwd_plan, _wgrad_plan


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--tile", type=int, default=-1)
    ap.add_argument("--splits", type=int, default=-1)
    ap.add_argument("--wsplits", type=int, default=-1, help="override the wgrad split count")
    ap.add_argument("--occupy", type=int, default=0,
                    help="hold R CUs with RCCL-sized workgroups on a side stream while timing (testing/diag.hip)")
    ap.add_argument("--dtile", type=int, default=-1, help="override the dgrad tile")
    ap.add_argument("--dsplits", type=int, default=-1, help="override the dgrad split count")
    ap.add_argument("--stages", default="3,0", help="fwd,wgrad LDS ring depth (wgrad: 0, the per-tile default)")
    ap.add_argument("--wtile", type=int, default=-1, help="override the wgrad tile (1 64x64, 2 128x128)")
    ap.add_argument("--waves", type=int, default=8, help="waves per workgroup of the fwd/dgrad kernel (4 or 8)")
    ap.add_argument("--region", type=int, default=1, help="1: tap-reuse (LDS-resident region) fwd/dgrad kernel")
    ap.add_argument("--rstages", type=int, default=0, help="region kernel B-ring stages (0 = max that fits)")
    ap.add_argument("--rwaves", type=int, default=8, help="region kernel waves per workgroup (4 or 8)")
    ap.add_argument("--fpf", type=int, default=1, help="streaming fwd/dgrad fragment prefetch (>= 3 stages)")
    a = ap.parse_args()
    C = _native.native()
    fs, ws = (int(v) for v in a.stages.split(","))
    C.set_conv_stages(fs, ws)
    C.set_conv_waves(a.waves)
    C.set_conv_region(a.region)
    C.set_conv_region_stages(a.rstages)
    C.set_conv_region_waves(a.rwaves)
    print(f"# stages fwd={fs} wgrad={ws} region={a.region}")
    dev = torch.device("cuda")
    def cur():  # current-stream handle at call time (graph capture switches streams)
        return torch.cuda.current_stream().cuda_stream
    B = a.batch
    layers = [(32, 8, 64), (16, 64, 128), (8, 128, 256), (4, 256, 512)]
    slab = torch.empty(64 * 1024 * 1024, device=dev)
    stats = torch.empty(4096 * 2 * 512, device=dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for li, (H, cin, cout) in enumerate(layers):
        M, K = B * H * H, 25 * cin
        # convolution inputs are zero-bordered [B, H+4, W+4, C] (the kernels' layout)
        x = torch.nn.functional.pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
        w = (torch.randn(cout, 5, 5, cin, device=dev) * 0.05).to(torch.bfloat16)
        y = torch.empty(B, H, H, cout, dtype=torch.bfloat16, device=dev)
        dy = torch.nn.functional.pad(torch.randn(B, H, H, cout, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
        wt = torch.empty(cin, 5, 5, cout, dtype=torch.bfloat16, device=dev)
        dx = torch.empty(B, H, H, cin, dtype=torch.bfloat16, device=dev)
        jobs = []
        t, sp = _fwd_plan(M, cout, K)
        if a.tile >= 0:
            t = a.tile
        if a.splits >= 0:
            sp = a.splits
        jobs.append((f"fwd{li+1}", 2 * M * cout * K, lambda t=t, sp=sp: C.conv_fwd(
            x.data_ptr(), w.data_ptr(), y.data_ptr(), stats.data_ptr(), slab.data_ptr(), B, H, H, cin, cout, 5, t,
            sp, cur()), f"tile{t} split{sp}"))
        if li > 0:
            dt, ds = _fwd_plan(M, cin, 25 * cout)
            if a.dtile >= 0:
                dt = a.dtile
            if a.dsplits >= 0:
                ds = a.dsplits
            jobs.append((f"dgrad{li+1}", 2 * M * cout * K, lambda dt=dt, ds=ds: C.conv_fwd(
                dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, slab.data_ptr(), B, H, H, cout, cin, 5, dt, ds,
                cur()),
                f"tile{dt} split{ds}"))
        wtile, wsp = _wgrad_plan(cout, K, M)
        if a.wtile >= 0 and cout % (128 if a.wtile == 2 else 64) == 0:
            wtile = a.wtile
            bm, bn = {2: (128, 128)}.get(wtile, (64, 64))
            tiles = (cout // bm) * ((K + bn - 1) // bn)
            wsp = 1
            while tiles * wsp < 256 and M // (wsp * 2) >= 2048:
                wsp *= 2
        if a.wsplits > 0:
            wsp = a.wsplits
        jobs.append((f"wgrad{li+1}", 2 * M * cout * K, lambda wtile=wtile, wsp=wsp: C.conv_wgrad(
            dy.data_ptr(), x.data_ptr(), slab.data_ptr(), B, H, H, cin, cout, 5, wsp, K, wtile, 0, cur()),
            f"tile{wtile} split{wsp}"))
        occ_stream = torch.cuda.Stream()
        for name, flops, fn, desc in jobs:
            if a.only and a.only not in name:
                continue
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            # replay a captured graph of `iters` launches: GPU time, not host launch rate
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for _ in range(a.iters):
                    fn()
            g.replay()
            torch.cuda.synchronize()
            if a.occupy:
                _native_testing().occupy_cus(a.occupy, 300000, 0, occ_stream.cuda_stream)
                torch.cuda._sleep(2_000_000)
            ev0.record()
            g.replay()
            ev1.record()
            torch.cuda.synchronize()
            us = ev0.elapsed_time(ev1) * 1e3 / a.iters
            print(f"{name:8s} M={M:6d} N={cout if 'dgrad' not in name else cin:4d} K={K:6d} {desc:16s} "
                  f"{us:8.2f} us  {flops / us / 1e6:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
