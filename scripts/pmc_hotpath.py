#!/usr/bin/env python3
"""Driver for the PMC-counter pass over the framework's hot kernels
(scripts/pmc_hotpath.sh): the fused SGD update, the sum-and-normalise scale
and the elastic-averaging step over a ResNet-50-sized flat buffer (25.6M
fp32), the 1x1-conv MFMA GEMMs (forward with BN statistics, dgrad, wgrad)
and the fused BatchNorm kernels at ResNet-50 batch-256 shapes.  Each runs
``--iters`` times."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.ops import flat as F
    from torch_distlearn_amd.ops.conv import _plan_1x1, _wgrad_plan

    C = _native.native()
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    n = 25_600_000
    p, g, mom, c, out = (torch.randn(n, device=dev) for _ in range(5))
    p16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    slot = torch.tensor([2.0, 0, 0, 0], device=dev)
    jobs = {
        "sgd": lambda: F.sgd_update_(p, g, 0.01, slot=slot, mom=mom, momentum=0.9, weight_decay=5e-4, shadow=p16),
        "scale": lambda: F.scale_by_count_(g, slot),
        "elastic": lambda: F.elastic_step_(p, c, out, 0.2, pending=mom, shadow=p16),
    }
    N, hw, cin, cout = 256, 56, 64, 256
    M = N * hw * hw
    x = torch.randn(M, cin, device=dev).to(torch.bfloat16)
    w = (torch.randn(cout, cin, device=dev) * 0.05).to(torch.bfloat16)
    wt = w.t().contiguous()
    y = torch.empty(M, cout, dtype=torch.bfloat16, device=dev)
    dy = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    dx = torch.empty(M, cin, dtype=torch.bfloat16, device=dev)
    ft, _ = _plan_1x1(M, cout, cin)
    dt, _ = _plan_1x1(M, cin, cout)
    rows = torch.empty((M + 127) // 128, 2, cout, device=dev)
    wtile, wsp = _wgrad_plan(cout, cin, M)
    wslab = torch.empty(wsp * cout * cin, device=dev)
    gw = torch.zeros(cout, cin, device=dev)
    jobs["conv_fwd_stats"] = lambda: C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), rows.data_ptr(), 0, M, 1, 1,
                                                 cin, cout, 1, ft, 1, s)
    jobs["conv_dgrad"] = lambda: C.conv_fwd(dy.data_ptr(), wt.data_ptr(), dx.data_ptr(), 0, 0, M, 1, 1, cout, cin, 1,
                                            dt, 1, s)
    jobs["conv_wgrad"] = lambda: (C.conv_wgrad(dy.data_ptr(), x.data_ptr(), wslab.data_ptr(), M, 1, 1, cin, cout, 1,
                                               wsp, cin, wtile, 0, s),
                                  C.slab_reduce_add(wslab.data_ptr(), gw.data_ptr(), wsp, cout, 1, cin, cin, s))
    acc = torch.zeros(4 * cout, device=dev)
    bw, bb = torch.ones(cout, device=dev), torch.zeros(cout, device=dev)
    save = torch.empty(2 * cout, device=dev)
    res = torch.randn(M, cout, device=dev).to(torch.bfloat16)
    dres = torch.empty_like(res)
    dwb, dbb = torch.empty(cout, device=dev), torch.empty(cout, device=dev)
    jobs["bn_fwd"] = lambda: C.bn_nhwc_fwd(y.data_ptr(), res.data_ptr(), dy.data_ptr(), acc.data_ptr(), bw.data_ptr(),
                                           bb.data_ptr(), save.data_ptr(), 0, 0, M, cout, 1e-5, 0.1, 1, 0, s)
    jobs["bn_bwd"] = lambda: C.bn_nhwc_bwd(dy.data_ptr(), y.data_ptr(), y.data_ptr(), save.data_ptr(), bw.data_ptr(),
                                           bb.data_ptr(), acc[2 * cout:].data_ptr(), res.data_ptr(), dres.data_ptr(),
                                           dwb.data_ptr(), dbb.data_ptr(), M, cout, 1, s)
    for name, fn in jobs.items():
        if a.only and a.only not in name:
            continue
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        print(name, "done", flush=True)


if __name__ == "__main__":
    main()
