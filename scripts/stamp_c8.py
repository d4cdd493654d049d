"""Debug: per-workgroup s_memtime phase stamps of the first-layer conv
(conv_fwd_c8_kernel, batch B): kernel entry, DMA landed, MFMA loop done, end.
    python scripts/stamp_c8.py [batch]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native

C = _native.native()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
H, cin, cout = 32, 8, 64
dev = torch.device("cuda")
x = torch.nn.functional.pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
w = (torch.randn(cout, 5, 5, cin, device=dev) * 0.05).to(torch.bfloat16)
y = torch.empty(B, H, H, cout, dtype=torch.bfloat16, device=dev)
rows = C.conv_fwd_stat_rows(B, H, H, cin, cout, 5, 2, 1)
stats = torch.zeros(max(rows, 4096), 2, cout, device=dev)
nwg = B * H * H // 128
dbg = torch.zeros(nwg * 4, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
for rep in range(6):
    C.set_conv_debug(dbg.data_ptr() if rep == 5 else 0)
    C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats.data_ptr(), 0, B, H, H, cin, cout, 5, 2, 1, s)
torch.cuda.synchronize()
C.set_conv_debug(0)
d = dbg.view(nwg, 4).cpu().double()
t0 = d[:, 0].min()
d = d - t0
# s_memtime runs at the shader clock (MHz): print cycles and the share of the span
span = float(d[:, 3].max())
q = lambda v: [round(float(v.quantile(p)), 0) for p in (0.0, 0.5, 0.9, 1.0)]  # noqa: E731
print(f"workgroups {nwg}, span {span:.0f} cycles")
print("start time        min/med/p90/max", q(d[:, 0]))
print("dma (start->land) min/med/p90/max", q(d[:, 1] - d[:, 0]))
print("mfma loop         min/med/p90/max", q(d[:, 2] - d[:, 1]))
print("epilogue          min/med/p90/max", q(d[:, 3] - d[:, 2]))
print("end time          min/med/p90/max", q(d[:, 3]))
