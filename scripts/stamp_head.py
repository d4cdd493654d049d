"""Phase stamps of the CIFAR head kernel (needs a DISTLEARN_CFLAGS=-DDL_HEAD_STAMPS
build): thread 0 of each of the B blocks records s_memtime at: 0 start, 1 BN
coefficients derived (bn_fin_block), 2 logits partials reduced, 3 after the
barrier, 4 after the softmax barrier, 5 dh stored, 6 RED LDS barrier, 7 end."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29541")
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
                         max_batch=B, graph=False)
for _ in range(3):
    tr.step(x, y)
torch.cuda.synchronize()
st = torch.zeros(B * 8, dtype=torch.int64, device=dev)
C.set_head_stamps(st.data_ptr())
tr.step(x, y)
torch.cuda.synchronize()
C.set_head_stamps(0)
d = st.view(B, 8).cpu().double()
t0 = d[:, 0].min()
names = ["fin", "logits", "barrier", "softmax", "dh", "red-lds", "atomics"]
print("phase means (cycles): " + "  ".join(f"{n} {(d[:, k + 1] - d[:, k]).mean():.0f}" for k, n in enumerate(names)))
print(f"block lifetime mean {(d[:, 7] - d[:, 0]).mean():.0f}, start spread {(d[:, 0] - t0).max():.0f}, "
      f"kernel span {(d[:, 7].max() - t0):.0f} cycles")
