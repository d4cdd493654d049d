#!/usr/bin/env python3
"""ResNet-50 BatchNorm(+ReLU/+residual) HIP kernels at batch 256: time and
achieved HBM GB/s of the statistics pass, the forward apply, and the backward
(reduce + apply), per shape.  One JSON line per shape."""
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

    C_ = _native.native()
    if "BN_RB" in os.environ:  # row-block cap of the statistics / backward-reduce kernels
        C_.set_bn_reduce_blocks(int(os.environ["BN_RB"]))
    tune = os.environ.get("BN_TUNE", "")  # "apply_rows,reduce_threads", e.g. 2,256 (round 2) / 4,1024
    if tune:
        C_.set_bn_tuning(*[int(v) for v in tune.split(",")])
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream().cuda_stream
    N = int(os.environ.get("BATCH", "256"))
    # (H, C, relu mode, residual): b1/b2 (relu, mask from x), b3 (+res, mask from y), down (no relu)
    shapes = [(112, 64, 2, False), (56, 64, 2, False), (56, 256, 1, True), (56, 256, 0, False), (28, 128, 2, False),
              (28, 512, 1, True), (14, 256, 2, False), (14, 1024, 1, True), (7, 512, 2, False), (7, 2048, 1, True)]
    for H, C, relu, res in shapes:
        M = N * H * H
        x = torch.randn(M, C, device=dev).to(torch.bfloat16)
        r = torch.randn(M, C, device=dev).to(torch.bfloat16) if res else None
        y = torch.empty_like(x)
        dy = torch.randn(M, C, device=dev).to(torch.bfloat16)
        dx = torch.empty_like(x)
        dres = torch.empty_like(x) if res else None
        acc = torch.zeros(4 * C, device=dev)
        w = torch.rand(C, device=dev) + 0.5
        b = torch.randn(C, device=dev) * 0.1
        save = torch.empty(2 * C, device=dev)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        dw, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        rp = r.data_ptr() if res else 0

        def fwd(stats):
            if not stats:
                acc[:2 * C].zero_()
            C_.bn_nhwc_fwd(x.data_ptr(), rp, y.data_ptr(), acc.data_ptr(), w.data_ptr(), b.data_ptr(),
                           save.data_ptr(), rm.data_ptr(), rv.data_ptr(), M, C, 1e-5, 0.1, int(relu > 0),
                           int(stats), s)

        def bwd():
            acc[2 * C:].zero_()
            C_.bn_nhwc_bwd(dy.data_ptr(), y.data_ptr() if relu == 1 else 0, x.data_ptr(), save.data_ptr(),
                           w.data_ptr(), b.data_ptr(), acc[2 * C:].data_ptr(), dx.data_ptr(),
                           dres.data_ptr() if res else 0, dw.data_ptr(), db.data_ptr(), M, C, relu, s)

        def bwd_apply():
            C_.bn_nhwc_bwd_pad(dy.data_ptr(), y.data_ptr() if relu == 1 else 0, x.data_ptr(), save.data_ptr(),
                               w.data_ptr(), b.data_ptr(), acc[2 * C:].data_ptr(), dx.data_ptr(),
                               dres.data_ptr() if res else 0, dw.data_ptr(), db.data_ptr(), M, C, relu, 1, 1, 0,
                               s, 1)

        z = timeit(lambda: acc.zero_())
        t_full = timeit(lambda: fwd(False)) - z
        t_apply = timeit(lambda: fwd(True))
        t_bwd = timeit(bwd) - z
        t_bapply = timeit(bwd_apply)
        E = M * C * 2  # bytes of one bf16 activation
        out = {"H": H, "C": C, "relu": relu, "res": res, "M": M,
               "stats_us": round(t_full - t_apply, 1), "stats_GBs": round(E / max(t_full - t_apply, 1e-3) / 1e3),
               "fwd_apply_us": round(t_apply, 1), "fwd_apply_GBs": round(E * (3 if res else 2) / t_apply / 1e3),
               "bwd_us": round(t_bwd, 1), "bwd_apply_us": round(t_bapply, 1),
               "bwd_apply_GBs": round(E * (2 + (relu == 1) + 1 + res) / t_bapply / 1e3),
               "bwd_reduce_GBs": round(E * (2 + (relu == 1)) / max(t_bwd - t_bapply, 1e-3) / 1e3),
               "bwd_GBs": round(E * ((2 + (relu == 1)) + (3 + (relu == 1) + res)) / t_bwd / 1e3)}
        out["tune"] = tune or "default"
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
