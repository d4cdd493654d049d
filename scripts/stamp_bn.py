"""Phase stamps of the fused BN forward (fin) / backward-apply kernels of the
CIFAR step (needs a DISTLEARN_CFLAGS=-DDL_BN_STAMPS build): per block thread 0
at start / after the coefficient prologue / end; per launch (C = 64, 128, 256):
block count, mean block lifetime and prologue, the spread of block start times
and the kernel span, in cycles."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29543")
import torch

from torch_distlearn_amd import Tree, _native
from torch_distlearn_amd.engine import DataParallelTrainer
from torch_distlearn_amd.models import CifarConvNet

C = _native.native()
dev = torch.device("cuda", 0)
tree = Tree(1, 1, host="127.0.0.1", port=int(os.environ["MASTER_PORT"]), device=dev)
B = 128
x = torch.randn(B, 32, 32, 3, device=dev).to(torch.bfloat16)
y = torch.randint(0, 10, (B,), device=dev)
tr = DataParallelTrainer(CifarConvNet(seed=0).to(dev), tree, lr=0.05, backend="hip", compute_dtype=torch.bfloat16,
                         max_batch=B, graph=True)
for _ in range(4):
    tr.step(x, y)
torch.cuda.synchronize()
st = torch.zeros(2 * 4 * 2048 * 4, dtype=torch.int64, device=dev)
C.set_bn_stamps(st.data_ptr())
tr._graph = None  # recapture with the stamp pointer live (a device global: read at run time anyway)
tr.step(x, y)
tr.step(x, y)
torch.cuda.synchronize()
C.set_bn_stamps(0)
d = st.view(2, 4, 2048, 4).cpu().double()
for kind, name in ((0, "fwd_fin"), (1, "bwd_apply")):
    for ci, Cc in enumerate((64, 128, 256)):
        e = d[kind, ci]
        n = int((e[:, 0] > 0).sum())
        if n == 0:
            continue
        e = e[:n]
        t0, t1 = e[:, 0].min(), e[:, 2].max()
        print(f"{name} C={Cc}: blocks {n}, life {(e[:, 2] - e[:, 0]).mean():.0f}, prologue {(e[:, 1] - e[:, 0]).mean():.0f}, "
              f"start spread {(e[:, 0] - t0).max():.0f}, span {t1 - t0:.0f} cycles", flush=True)
