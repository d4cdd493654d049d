"""ResNet-50 (BASELINE config 5) on CPU: shapes / parameter count, the fused
BN+act fallback path equals act(BN(x) [+ r]) of plain PyTorch ops, and the
HIP BN op's host-side shape guard."""
import pytest
import torch
import torch.nn.functional as F


def test_resnet50_shapes_and_params():
    from torch_distlearn_amd.models import ResNet50

    m = ResNet50(seed=0)
    n = sum(p.numel() for p in m.parameters())
    assert n == 25557032  # torchvision resnet50: 25,557,032 parameters
    y = m(torch.randn(2, 64, 64, 3))
    assert y.shape == (2, 1000) and torch.allclose(y.exp().sum(1), torch.ones(2), atol=1e-4)


@pytest.mark.parametrize("relu,res", [(True, False), (True, True), (False, False)])
def test_bn_act_fallback_matches_torch(relu, res):
    from torch_distlearn_amd.models.resnet import _BN

    torch.manual_seed(0)
    bn = _BN(16)
    bn.weight.data.uniform_(0.5, 1.5)
    x = torch.randn(4, 16, 5, 5)
    r = torch.randn(4, 16, 5, 5) if res else None
    got = bn.act(x, relu=relu, residual=r)
    want = F.batch_norm(x, torch.zeros(16), torch.ones(16), bn.weight, bn.bias, True, 0.1, 1e-5)
    want = want + r if r is not None else want
    want = F.relu(want) if relu else want
    assert torch.allclose(got, want, atol=1e-5)


def test_bn_nhwc_supported_guard():
    from torch_distlearn_amd.ops.bn_nhwc import bn_act, supported

    x = torch.randn(2, 64, 4, 4)
    assert not supported(x)  # CPU fp32
    with pytest.raises(ValueError):
        bn_act(x, torch.ones(64), torch.zeros(64), None, None)
