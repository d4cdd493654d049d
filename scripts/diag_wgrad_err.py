"""Where do wrong weight-gradient elements lie (tile 1, shape (3, 8, 16, 64))?
Prints the error structure by output channel, tap and input channel."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from torch_distlearn_amd import _native

C = _native.native()
dev = torch.device("cuda")
s = torch.cuda.current_stream().cuda_stream
B, H, cin, cout = 3, 8, 16, 64
g = torch.Generator(device=dev).manual_seed(11 + B * H + cout)
x = torch.randn(B, H, H, cin, device=dev, generator=g).to(torch.bfloat16)
w = (torch.randn(cout, 5, 5, cin, device=dev, generator=g) * 0.05).to(torch.bfloat16)
dy = torch.randn(B, H, H, cout, device=dev, generator=g).to(torch.bfloat16)
xr = x.float().permute(0, 3, 1, 2).requires_grad_(True)
wr = w.float().permute(0, 3, 1, 2).requires_grad_(True)
F.conv2d(xr, wr, padding=2).backward(dy.float().permute(0, 3, 1, 2))
ref = wr.grad.permute(0, 2, 3, 1)
K = 25 * cin
xp, dyp = F.pad(x, (0, 0, 2, 2, 2, 2)), F.pad(dy, (0, 0, 2, 2, 2, 2))
print("ptrs", hex(xp.data_ptr()), hex(dyp.data_ptr()))
for tile in (1,):
    slabs = torch.full((1, cout, K), float("nan"), device=dev)
    C.conv_wgrad(dyp.data_ptr(), xp.data_ptr(), slabs.data_ptr(), B, H, H, cin, cout, 5, 1, K, tile, 0, s)
    torch.cuda.synchronize()
    dw = slabs[0].view(cout, 25, cin)
    r = ref.reshape(cout, 25, cin)
    bad = (dw - r).abs() > 1e-3 * r.abs().max()
    print(f"tile {tile}: {int(bad.sum())} bad of {bad.numel()}; nan {int(torch.isnan(dw).sum())}")
    if bad.any():
        print(" bad co:", torch.nonzero(bad.any(2).any(1)).flatten().tolist()[:64])
        print(" bad taps:", torch.nonzero(bad.any(2).any(0)).flatten().tolist())
        print(" bad ci:", torch.nonzero(bad.any(0).any(0)).flatten().tolist())
        kk = torch.nonzero(bad.any(0).reshape(-1)).flatten()
        print(" bad k (tap*16+ci) min/max:", int(kk.min()), int(kk.max()), "count", kk.numel())
        i = torch.nonzero(bad)[0].tolist()
        print(" first bad", i, float(dw[tuple(i)]), float(r[tuple(i)]))
