"""Debug: executor backward with the fused split-K combine + BN backward reduce
(DISTLEARN_FUSE_COMBINE=1) vs separate launches, reduction mode 0: per-layer
differences of dP and of every gradient tensor."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["DISTLEARN_REDUCE_ATOMIC"] = "0"
import torch  # noqa: E402

from torch_distlearn_amd import FlatParams  # noqa: E402
from torch_distlearn_amd.models import CifarConvNet  # noqa: E402
from torch_distlearn_amd.models.cifar_hip import CifarHIPExecutor  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(6)
x = torch.randn(B, 32, 32, 3, device=dev, generator=g).to(torch.bfloat16)
y = torch.randint(0, 10, (B,), device=dev, generator=g)
res = []
for fuse in ("0", "1", "0", "1"):
    os.environ["DISTLEARN_FUSE_COMBINE"] = fuse
    mdl = CifarConvNet(seed=4).to(dev)
    flat = FlatParams(mdl, grads=True, shadow_bf16=True)
    ex = CifarHIPExecutor(mdl, flat, max_batch=B)
    ex.forward_backward(x.contiguous(), y)
    torch.cuda.synchronize()
    res.append(([d.clone() for d in ex.dP], [v.clone() for v in flat.views_of(flat.grad)], ex.dgrad_plan))
print("dgrad plans", res[0][2])
for k, (a, b) in enumerate([(0, 2), (1, 3), (0, 1)]):
    print(["unfused vs unfused", "fused vs fused", "unfused vs fused"][k])
    for i, (p, q) in enumerate(zip(res[a][0], res[b][0])):
        print(f"  dP[{i}] max|diff| {float((p.float() - q.float()).abs().max()):.3e}  equal {torch.equal(p, q)}")
    for i, (p, q) in enumerate(zip(res[a][1], res[b][1])):
        if not torch.equal(p, q):
            print(f"  grad leaf {i} {tuple(p.shape)} max|diff| {float((p - q).abs().max()):.3e}")
