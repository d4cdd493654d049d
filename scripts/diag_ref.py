"""Is the MIOpen fp32 reference the culprit?  Compare torch GPU fp32 conv
backward-weights against CPU fp64 on the failing shape, after running the
same sequence of GPU work the test runs first."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

dev = torch.device("cuda")
for (B, H, cin, cout) in [(8, 32, 8, 64), (8, 16, 64, 128), (8, 8, 128, 256), (32, 4, 256, 512), (3, 8, 16, 64)]:
    g = torch.Generator(device=dev).manual_seed(11 + B * H + cout)
    x = torch.randn(B, H, H, cin, device=dev, generator=g).to(torch.bfloat16)
    w = (torch.randn(cout, 5, 5, cin, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    dy = torch.randn(B, H, H, cout, device=dev, generator=g).to(torch.bfloat16)
    refs = []
    for d, dt in ((dev, torch.float32), ("cpu", torch.float64)):
        xr = x.to(d, dt).permute(0, 3, 1, 2).requires_grad_(True)
        wr = w.to(d, dt).permute(0, 3, 1, 2).requires_grad_(True)
        F.conv2d(xr, wr, padding=2).backward(dy.to(d, dt).permute(0, 3, 1, 2))
        refs.append((xr.grad.double().cpu(), wr.grad.double().cpu()))
    rx = float((refs[0][0] - refs[1][0]).norm() / refs[1][0].norm())
    rw = float((refs[0][1] - refs[1][1]).norm() / refs[1][1].norm())
    print(f"{(B, H, cin, cout)}: MIOpen fp32 vs CPU fp64: dgrad rel {rx:.2e}, wgrad rel {rw:.2e}", flush=True)
