"""Phase stamps of the weight-gradient kernel (needs a DISTLEARN_CFLAGS=
-DDL_WGRAD_STAMPS build): per workgroup, waves 0 and NW-1 record s_memtime at
start / loop begin / loop end / end and the summed cycles of every K step's
wait (vmcnt + barrier) and issue work (fragment reads, DMA issue, MFMAs).
Run on the CIFAR layer shapes of scripts/bench_conv.py."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native
from torch_distlearn_amd.models.cifar_hip import _wgrad_plan

C = _native.native()
dev = torch.device("cuda")
B = 128
order = int(os.environ.get("WORDER", "1"))
C.set_conv_wgrad_order(order)
slab = torch.empty(64 * 1024 * 1024, device=dev)
st = torch.zeros(4096 * 2 * 6, dtype=torch.int64, device=dev)
s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
print(f"# wgrad order {order}; cycles (s_memtime), mean over workgroups [wave0 / last wave]")
for li, (H, cin, cout) in enumerate([(32, 8, 64), (16, 64, 128), (8, 128, 256), (4, 256, 512)]):
    M, K = B * H * H, 25 * cin
    x = torch.nn.functional.pad(torch.randn(B, H, H, cin, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
    dy = torch.nn.functional.pad(torch.randn(B, H, H, cout, device=dev), (0, 0, 2, 2, 2, 2)).to(torch.bfloat16)
    wtile, wsp = _wgrad_plan(cout, K, M)
    run = lambda: C.conv_wgrad(dy.data_ptr(), x.data_ptr(), slab.data_ptr(), B, H, H, cin, cout, 5, wsp, K,  # noqa
                               wtile, 0, s())
    for _ in range(3):
        run()
    torch.cuda.synchronize()
    st.zero_()
    C.set_conv_wgrad_stamps(st.data_ptr())
    run()
    torch.cuda.synchronize()
    C.set_conv_wgrad_stamps(0)
    d = st.view(-1, 2, 6).cpu().double()
    n = int((d[:, 0, 0] > 0).sum())
    d = d[:n]
    t0 = d[:, :, 0].min()
    span = d[:, :, 5].max() - t0
    for w in (0, 1):
        e = d[:, w]
        life = (e[:, 5] - e[:, 0]).mean()
        pro = (e[:, 1] - e[:, 0]).mean()
        loop = (e[:, 4] - e[:, 1]).mean()
        wait = e[:, 2].mean()
        work = e[:, 3].mean()
        epi = (e[:, 5] - e[:, 4]).mean()
        startspread = (e[:, 0] - t0).max()
        print(f"wgrad{li + 1} tile{wtile} split{wsp} wgs={n} wave{'0' if w == 0 else 'L'}: span {span:8.0f} "
              f"life {life:7.0f} prologue {pro:6.0f} loop {loop:7.0f} (wait {wait:7.0f} work {work:7.0f}) "
              f"epilogue {epi:6.0f} last-start {startspread:7.0f}", flush=True)
