"""Debug: per-workgroup s_memtime stamps of one conv_fwd launch (fwd2 shape).
Prints distributions of (setup, loop, epilogue) durations and start skew."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native

C = _native.native()
ab = int(sys.argv[1]) if len(sys.argv) > 1 else 0
B, H, cin, cout = 128, 16, 64, 128
dev = torch.device("cuda")
x = torch.nn.functional.pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)  # zero border
w = (torch.randn(cout, 5, 5, cin, device=dev) * 0.05).to(torch.bfloat16)
y = torch.empty(B, H, H, cout, dtype=torch.bfloat16, device=dev)
stats = torch.empty(4096 * 2 * cout, device=dev)
dbg = torch.zeros(256 * 4, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
C.set_conv_waves(ab if ab in (4, 8) else 4)
for rep in range(3):
    C.set_conv_debug(dbg.data_ptr() if rep == 2 else 0)
    C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats.data_ptr(), 0, B, H, H, cin, cout, 5, 0, 1, s)
torch.cuda.synchronize()
C.set_conv_debug(0)
d = dbg.view(256, 4).cpu().double()
t0 = d[:, 0].min()
st, su, lo, en = d[:, 0] - t0, d[:, 1] - d[:, 0], d[:, 2] - d[:, 1], d[:, 3] - d[:, 2]
q = lambda v: f"min {v.min():8.0f} med {v.median():8.0f} max {v.max():8.0f}"  # noqa: E731
print(f"waves={ab} (cycles of s_memtime)")
print(" start skew ", q(st))
print(" setup      ", q(su))
print(" k-loop     ", q(lo))
print(" epilogue   ", q(en))
print(" total span ", float((d[:, 3].max() - t0)))
