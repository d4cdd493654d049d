"""The ResNet-50 operations that left MIOpen / hipBLAS this round (ops/conv.py
StemConv / Conv1x1S2 / Conv3x3S2, ops/head.py ResNetHeadNLL) against fp32
PyTorch references of the same ops: forward, input gradient and the fp32
weight gradient written into the flat gradient."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
CL = torch.channels_last
BF = torch.bfloat16


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from torch_distlearn_amd import _native

    _native.native().set_reduce_atomic(0)
    return torch.device("cuda", 0)


def _ref(x, w16, go, stride, pad):
    xr, wr = x.float().detach().requires_grad_(True), w16.float().detach().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, pad)
    yr.backward(go.float())
    return yr, xr.grad, wr.grad


@pytest.mark.parametrize("N,H", [(2, 224), (3, 64), (2, 30)])
def test_stem_conv_matches_fp32(dev, N, H):
    from torch_distlearn_amd.ops.conv import ShadowBinding, StemConv

    g = torch.Generator(device=dev).manual_seed(H)
    x = torch.randn(N, 3, H, H, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    w16 = (torch.randn(64, 3, 7, 7, device=dev, generator=g) * (3 * 49) ** -0.5).to(BF)
    prior = torch.randn(64, 3, 7, 7, device=dev, generator=g)
    g32 = prior.clone()
    ready = []
    bind = ShadowBinding(w16.view(-1), g32.view(-1), lambda: ready.append(1))
    stats = torch.zeros(128, device=dev)
    y = StemConv.apply(x, torch.nn.Parameter(w16.float()), bind, stats)
    go = torch.randn_like(y)
    y.backward(go)
    yr, _, wg = _ref(x, w16, go, 2, 3)
    torch.cuda.synchronize()
    assert y.shape == yr.shape and y.is_contiguous(memory_format=CL)
    assert _rel(y, yr) < 1e-2
    assert _rel(g32 - prior, wg) < 1e-2 and ready == [1]
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, 64)
    torch.testing.assert_close(stats[:64], yf.sum(0), rtol=1e-3, atol=1e-1)


@pytest.mark.parametrize("N,cin,H,cout", [(2, 256, 56, 512), (3, 512, 28, 1024), (2, 1024, 14, 2048), (2, 64, 8, 128)])
def test_conv1x1_s2_matches_fp32(dev, N, cin, H, cout):
    from torch_distlearn_amd.ops.conv import Conv1x1S2, ShadowBinding

    g = torch.Generator(device=dev).manual_seed(cin + H)
    x = torch.randn(N, cin, H, H, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    w16 = (torch.randn(cout, cin, 1, 1, device=dev, generator=g) * cin ** -0.5).to(BF)
    g32 = torch.zeros(cout, cin, device=dev)
    bind = ShadowBinding(w16.view(cout, cin), g32, lambda: None)
    xi = x.detach().requires_grad_(True)
    y = Conv1x1S2.apply(xi, torch.nn.Parameter(w16.float()), bind, None)
    go = torch.randn_like(y)
    y.backward(go)
    yr, dxr, wg = _ref(x, w16, go, 2, 0)
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-2 and _rel(xi.grad, dxr) < 1e-2 and _rel(g32, wg.view(cout, cin)) < 1e-2


def test_conv1x1_s2_dgrad_accumulates_into_c1(dev):
    """The downsample's input gradient handed to the stride-1 1x1 conv that
    shares its input: c1's backward adds it in place at the even pixels."""
    from torch_distlearn_amd.ops.conv import Conv1x1, Conv1x1S2, ShadowBinding

    N, cin, H = 2, 256, 28
    g = torch.Generator(device=dev).manual_seed(11)
    x = torch.randn(N, cin, H, H, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    wa = (torch.randn(128, cin, 1, 1, device=dev, generator=g) * cin ** -0.5).to(BF)
    wd = (torch.randn(512, cin, 1, 1, device=dev, generator=g) * cin ** -0.5).to(BF)
    ba = ShadowBinding(wa.view(128, cin), torch.zeros(128, cin, device=dev), lambda: None)
    bd = ShadowBinding(wd.view(512, cin), torch.zeros(512, cin, device=dev), lambda: None)
    link = {}
    xi = x.detach().requires_grad_(True)
    ya = Conv1x1.apply(xi, torch.nn.Parameter(wa.float()), ba, None, link, None)
    yd = Conv1x1S2.apply(xi, torch.nn.Parameter(wd.float()), bd, None, link)
    ga, gd = torch.randn_like(ya), torch.randn_like(yd)
    (ya.float() * ga.float()).sum().add((yd.float() * gd.float()).sum()).backward()
    xr = x.float().detach().requires_grad_(True)
    (F.conv2d(xr, wa.float()) * ga.float()).sum().add((F.conv2d(xr, wd.float(), stride=2) * gd.float()).sum()).backward()
    torch.cuda.synchronize()
    assert "s2" not in link
    assert _rel(xi.grad, xr.grad) < 1e-2


@pytest.mark.parametrize("N,cin,H,cout", [(2, 128, 56, 128), (2, 256, 28, 256), (2, 512, 14, 512), (3, 64, 10, 128)])
def test_conv3x3_s2_matches_fp32(dev, N, cin, H, cout):
    from torch_distlearn_amd.ops.conv import Conv3x3S2, ShadowBinding

    g = torch.Generator(device=dev).manual_seed(cin + 3 * H)
    x = torch.randn(N, cin, H, H, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    w16 = (torch.randn(cout, cin, 3, 3, device=dev, generator=g) * (9 * cin) ** -0.5).to(BF)
    bind = ShadowBinding(w16.view(-1), torch.zeros(cout * cin * 9, device=dev), lambda: None)
    bind.wcl = w16.contiguous(memory_format=CL)  # [Cout][3][3][Cin] in memory
    xi = x.detach().requires_grad_(True)
    y = Conv3x3S2.apply(xi, torch.nn.Parameter(w16.float()), bind, None)
    go = torch.randn_like(y)
    y.backward(go)
    yr, dxr, wg = _ref(x, w16, go, 2, 1)
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-2
    assert _rel(xi.grad, dxr) < 1e-2
    assert _rel(bind.g32.view(cout, cin, 3, 3), wg) < 1e-2


@pytest.mark.parametrize("B,C,ncls", [(64, 2048, 1000), (8, 256, 100), (256, 2048, 1000)])
def test_resnet_head_matches_fp32(dev, B, C, ncls):
    """mean + Linear + LogSoftMax + NLL forward and backward in one node
    against the fp32 autograd reference (bf16 operands, fp32 accumulation /
    softmax / gradients)."""
    from torch_distlearn_amd.ops.head import ResNetHeadNLL, head_supported

    g = torch.Generator(device=dev).manual_seed(B + ncls)
    h = torch.randn(B, C, 7, 7, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    w = torch.randn(ncls, C, device=dev, generator=g) * C ** -0.5
    b = torch.randn(ncls, device=dev, generator=g) * 0.1
    y = torch.randint(0, ncls, (B,), device=dev, generator=g)
    assert head_supported(h, ncls)
    gw, gb = torch.zeros(ncls, C, device=dev), torch.zeros(ncls, device=dev)
    ready = []
    hi = h.detach().requires_grad_(True)
    loss, logp = ResNetHeadNLL.apply(hi, torch.nn.Parameter(w), torch.nn.Parameter(b), y,
                                     (gw, gb, lambda: ready.append(1)))
    loss.backward()
    hr = h.float().detach().requires_grad_(True)
    wr, br = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
    lr_ = F.log_softmax(F.linear(hr.mean((2, 3)), wr, br), dim=1)
    Lr = F.nll_loss(lr_, y)
    Lr.backward()
    torch.cuda.synchronize()
    assert abs(float(loss) - float(Lr)) < 1e-2 * max(1.0, float(Lr))
    assert _rel(logp, lr_) < 1e-2
    assert _rel(hi.grad, hr.grad) < 2e-2
    assert _rel(gw, wr.grad) < 2e-2 and _rel(gb, br.grad) < 1e-3
    assert ready == [1]
    with torch.no_grad():
        _, lp_eval = ResNetHeadNLL.apply(h, w, b, None, None)
    assert _rel(lp_eval, lr_) < 1e-2


def test_resnet_head_honours_loss_scale_and_labels(dev):
    """the fused head's gradients follow d loss (a scaled loss
    scales every gradient), a loss built on the log-probabilities raises
    instead of training wrong, a second backward raises, int32 labels are
    refused and an out-of-range label gives a NaN loss."""
    from torch_distlearn_amd.ops.head import ResNetHeadNLL

    B, C, ncls = 8, 256, 100
    g = torch.Generator(device=dev).manual_seed(5)
    h = torch.randn(B, C, 7, 7, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    w = torch.randn(ncls, C, device=dev, generator=g) * C ** -0.5
    b = torch.randn(ncls, device=dev, generator=g) * 0.1
    y = torch.randint(0, ncls, (B,), device=dev, generator=g)

    def run(scale):
        gw, gb = torch.zeros(ncls, C, device=dev), torch.zeros(ncls, device=dev)
        hi = h.detach().requires_grad_(True)
        loss, _ = ResNetHeadNLL.apply(hi, torch.nn.Parameter(w), torch.nn.Parameter(b), y, (gw, gb, lambda: None))
        (loss * scale).backward()
        torch.cuda.synchronize()
        return hi.grad.float(), gw, gb

    d1, w1, b1 = run(1.0)
    d3, w3, b3 = run(3.0)
    assert _rel(d3, 3 * d1) < 1e-2 and _rel(w3, 3 * w1) < 1e-2 and _rel(b3, 3 * b1) < 1e-5
    hi = h.detach().requires_grad_(True)
    bind = (torch.zeros(ncls, C, device=dev), torch.zeros(ncls, device=dev), lambda: None)
    loss, logp = ResNetHeadNLL.apply(hi, torch.nn.Parameter(w), torch.nn.Parameter(b), y, bind)
    with pytest.raises(RuntimeError, match="not differentiable"):
        (loss + logp.sum()).backward()
    loss, _ = ResNetHeadNLL.apply(hi, torch.nn.Parameter(w), torch.nn.Parameter(b), y, bind)
    loss.backward(retain_graph=True)
    with pytest.raises(RuntimeError, match="twice"):
        loss.backward()
    with pytest.raises(ValueError, match="int64"):
        ResNetHeadNLL.apply(hi, torch.nn.Parameter(w), torch.nn.Parameter(b), y.int(), bind)
    bad = y.clone()
    bad[3] = ncls + 7
    with torch.no_grad():
        loss, _ = ResNetHeadNLL.apply(h, w, b, bad, bind)
    assert torch.isnan(loss).item()


def test_resnet50_step_has_no_vendor_convs(dev):
    """A ResNet-50 training step (batch 64, 64x64 images) dispatches no MIOpen
    convolution and no hipBLAS GEMM: every conv, the classifier and the loss
    run on the library's own kernels (torch.profiler kernel names)."""
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50

    tree = Tree(1, 1, host="127.0.0.1", port=29577, device=dev)
    model = ResNet50(num_classes=1000, seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.02, backend="torch", compute_dtype=BF, max_batch=64)
    tr.synchronize_parameters()
    x = torch.randn(64, 64, 64, 3, device=dev).to(BF)
    y = torch.randint(0, 1000, (64,), device=dev)
    tr.step(x, y)
    torch.cuda.synchronize()
    with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CUDA]) as prof:
        loss = tr.step(x, y)
        torch.cuda.synchronize()
    names = [e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA]
    bad = [n for n in names if any(k in n for k in ("igemm", "Cijk", "ck::", "naive_conv", "MIOpen", "miopen",
                                                   "grouped_conv", "SubTensorOp"))]
    assert not bad, sorted(set(bad))[:10]
    assert bool(torch.isfinite(loss))
