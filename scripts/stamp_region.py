"""Debug: per-workgroup s_memtime stamps of one region-kernel conv launch
(layer L of the CIFAR net, fwd or dgrad): issue / first-data / loop / epilogue.
    python scripts/stamp_region.py <layer 2..4> <fwd|dgrad> [ablate bits: 1 no DMA, 2 no MFMA]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native
from torch_distlearn_amd.models.cifar_hip import _fwd_plan

C = _native.native()
C.set_conv_region(int(os.environ.get("REGION", "1")))  # 2: whole-image tiles too (layers 3-4)
C.set_conv_region_ablate(int(sys.argv[3]) if len(sys.argv) > 3 else 0)
C.set_conv_region_stages(int(sys.argv[4]) if len(sys.argv) > 4 else 0)
C.set_conv_region_waves(int(sys.argv[5]) if len(sys.argv) > 5 else 8)
L = int(sys.argv[1])
mode = sys.argv[2]
B = 128
H, cin, cout = {2: (16, 64, 128), 3: (8, 128, 256), 4: (4, 256, 512)}[L]
if mode == "dgrad":
    cin, cout = cout, cin
dev = torch.device("cuda")
x = torch.nn.functional.pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
w = (torch.randn(cout, 5, 5, cin, device=dev) * 0.05).to(torch.bfloat16)
y = torch.empty(B, H, H, cout, dtype=torch.bfloat16, device=dev)
stats = torch.empty(4096 * 2 * cout, device=dev)
slab = torch.empty(16 * B * H * H * cout, device=dev)
t, sp = _fwd_plan(B * H * H, cout, 25 * cin)
ntiles = (B * H * H + 127) // 128 * (cout // (128 if t == 0 else 64)) * sp
dbg = torch.zeros(ntiles * 5, dtype=torch.int64, device=dev)
s = torch.cuda.current_stream().cuda_stream
for rep in range(4):
    C.set_conv_debug(dbg.data_ptr() if rep == 3 else 0)
    C.conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), stats.data_ptr() if mode == "fwd" else 0, slab.data_ptr(),
               B, H, H, cin, cout, 5, t, sp, s)
torch.cuda.synchronize()
C.set_conv_debug(0)
d = dbg.view(ntiles, 5).cpu().double()
t0 = d[:, 0].min()
q = lambda v: f"min {v.min():8.0f} med {v.median():8.0f} max {v.max():8.0f}"  # noqa: E731
print(f"layer {L} {mode} tile {t} splits {sp} ablate {sys.argv[3] if len(sys.argv) > 3 else 0} stages {sys.argv[4] if len(sys.argv) > 4 else 'max'} waves {sys.argv[5] if len(sys.argv) > 5 else 8}: {ntiles} workgroups (s_memtime cycles)")
print(" start skew    ", q(d[:, 0] - t0))
print(" issue         ", q(d[:, 1] - d[:, 0]))
print(" first data    ", q(d[:, 2] - d[:, 1]))
print(" k-loop        ", q(d[:, 3] - d[:, 2]))
print(" epilogue      ", q(d[:, 4] - d[:, 3]))
print(" total span    ", float((d[:, 4].max() - t0)))
