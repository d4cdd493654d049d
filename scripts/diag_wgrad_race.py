"""Repeat the 64x64 / 128x128 weight-gradient kernels on small test shapes and
count results that differ from the first run (bitwise: the kernel is
deterministic) and from fp32 -- per main-loop order (g_wgrad_order)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from torch_distlearn_amd import _native

C = _native.native()
dev = torch.device("cuda")
s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731


def pad(t):
    return F.pad(t, (0, 0, 2, 2, 2, 2))


for (B, H, cin, cout) in [(3, 8, 16, 64), (8, 16, 64, 128), (5, 4, 32, 128), (8, 8, 128, 256)]:
    g = torch.Generator(device=dev).manual_seed(11 + B * H + cout)
    x = torch.randn(B, H, H, cin, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, 5, 5, cin, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, H, H, cout, device=dev, generator=g).to(torch.bfloat16)
    xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
    wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
    F.conv2d(xr, wr, padding=2).backward(dy.float().permute(0, 3, 1, 2))
    dw_ref = wr.grad.permute(0, 2, 3, 1)
    K = 25 * cin
    xp, dyp = pad(x), pad(dy)
    for tile in (1, 2):
        if cout % (64 if tile == 1 else 128):
            continue
        for order in (0, 1):
            C.set_conv_wgrad_order(order)
            first, bad_bits, bad_ref, worst = None, 0, 0, 0.0
            for rep in range(40):
                slabs = torch.full((1, cout, K), float("nan"), device=dev)
                C.conv_wgrad(dyp.data_ptr(), xp.data_ptr(), slabs.data_ptr(), B, H, H, cin, cout, 5, 1, K, tile, 0, s())
                torch.cuda.synchronize()
                dw = slabs[0].view(cout, 5, 5, cin)
                rel = float((dw - dw_ref).norm() / dw_ref.norm())
                worst = max(worst, rel)
                bad_ref += rel > 1e-4
                if first is None:
                    first = dw.clone()
                elif not torch.equal(first, dw):
                    bad_bits += 1
            print(f"shape {(B, H, cin, cout)} tile {tile} order {order}: {bad_ref}/40 off fp32 (worst rel {worst:.2e}), "
                  f"{bad_bits}/39 differ from run 1", flush=True)
C.set_conv_wgrad_order(1)
