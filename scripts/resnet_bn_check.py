"""Numerics of the ResNet-50 BatchNorm modes on the GPU: the mixed (bf16 input,
fp32 statistics) kernel against an fp32 PyTorch reference of the same op,
forward output and input/weight gradients."""
import torch
import torch.nn.functional as F

torch.manual_seed(0)
dev = "cuda"
for shape in [(256, 64, 56, 56), (256, 2048, 7, 7)]:
    x32 = (torch.randn(shape, device=dev) * 3 + 1).contiguous(memory_format=torch.channels_last)
    xb = x32.to(torch.bfloat16)
    c = shape[1]
    w = torch.rand(c, device=dev) + 0.5
    b = torch.randn(c, device=dev)
    go = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = {}
    for mode in ("ref", "mixed"):
        xi = (xb.float() if mode == "ref" else xb).detach().requires_grad_(True)
        wi, bi = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        y = F.batch_norm(xi, rm, rv, wi, bi, True, 0.1, 1e-5)
        y.backward(go.to(y.dtype))
        outs[mode] = (y.float(), xi.grad.float(), wi.grad, bi.grad, rm, rv)
    names = ["y", "dx", "dw", "db", "running_mean", "running_var"]
    for n, a, r in zip(names, outs["mixed"], outs["ref"]):
        rel = float((a - r).norm() / (r.norm() + 1e-12))
        print(f"{shape} {n}: rel err {rel:.2e}")
        assert rel < 2e-2, (shape, n, rel)
print("bn check ok")
