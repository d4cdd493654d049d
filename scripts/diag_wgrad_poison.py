"""Does any conv kernel read LDS it did not write in its own launch?  Poison
every CU's LDS with NaN (bf16 pair 0x7FC07FC0) right before each launch and
compare with the unpoisoned result, per wgrad tile and shape."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F

from torch_distlearn_amd import _native

C = _native.native()
T = _native.testing()
dev = torch.device("cuda")
s = torch.cuda.current_stream().cuda_stream
for (B, H, cin, cout) in [(3, 8, 16, 64), (8, 32, 8, 64), (8, 16, 64, 128), (5, 4, 32, 128), (8, 8, 128, 256),
                          (32, 4, 256, 512)]:
    g = torch.Generator(device=dev).manual_seed(1 + B * H + cout)
    x = torch.randn(B, H, H, cin, device=dev, generator=g).to(torch.bfloat16)
    dy = torch.randn(B, H, H, cout, device=dev, generator=g).to(torch.bfloat16)
    xp, dyp = F.pad(x, (0, 0, 2, 2, 2, 2)), F.pad(dy, (0, 0, 2, 2, 2, 2))
    K = 25 * cin
    for tile in (0, 1, 2, 3, 4):
        if cout % {1: 64, 3: 256, 4: 256}.get(tile, 128) or (tile == 4 and H > 32):
            continue
        for splits in (1, 3):
            res = []
            for poison in (None, 0x7FC07FC0, 0x3F803F80):
                slabs = torch.zeros((splits, cout, K), device=dev)
                if poison is not None:
                    T.lds_poison(1024, poison, s)
                C.conv_wgrad(dyp.data_ptr(), xp.data_ptr(), slabs.data_ptr(), B, H, H, cin, cout, 5, splits, K, tile,
                             0, s)
                torch.cuda.synchronize()
                res.append(slabs.clone())
            same = [torch.equal(res[0], r) for r in res[1:]]
            nan = [int(torch.isnan(r).sum()) for r in res]
            print(f"shape {(B, H, cin, cout)} tile {tile} splits {splits}: poisoned == clean {same}, nan {nan}",
                  flush=True)
