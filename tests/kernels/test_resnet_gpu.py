"""ResNet-50 (BASELINE config 5) on the GPU: the mixed-precision BatchNorm
(bf16 activations, fp32 statistics; DISTLEARN_RESNET_BN=mixed, the default)
against an fp32 PyTorch reference of the same op, and one finite training
step of the model through the data-parallel trainer."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape", [(64, 64, 28, 28), (32, 2048, 7, 7)])
def test_bn_mixed_matches_fp32(shape):
    torch.manual_seed(0)
    dev = "cuda"
    xb = (torch.randn(shape, device=dev) * 3 + 1).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    c = shape[1]
    w, b = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev)
    go = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for x in (xb.float(), xb):
        xi = x.detach().requires_grad_(True)
        wi, bi = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        y = F.batch_norm(xi, rm, rv, wi, bi, True, 0.1, 1e-5)
        assert y.dtype == x.dtype
        y.backward(go.to(y.dtype))
        outs.append((y.float(), xi.grad.float(), wi.grad, bi.grad, rm, rv))
    for a, r in zip(outs[1], outs[0]):
        assert float((a - r).norm() / (r.norm() + 1e-12)) < 2e-2


def test_resnet50_train_step():
    import os

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29571, device=dev)
    model = ResNet50(num_classes=100, seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.02, backend="torch", compute_dtype=torch.bfloat16, max_batch=8)
    tr.synchronize_parameters()
    x = torch.randn(8, 64, 64, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 100, (8,), device=dev)
    before = tr.flat.data.clone()
    losses = [float(tr.step(x, y)) for _ in range(3)]
    torch.cuda.synchronize()
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert float((tr.flat.data - before).abs().max()) > 0
    tr.finish()
