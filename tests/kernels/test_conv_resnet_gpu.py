"""ResNet-50 convolutions on the shadow weights (ops/conv.py) against fp32
PyTorch references of the same ops: the stride-1 1x1 convolutions on the
hand-written MFMA kernels (forward, dgrad, fp32 wgrad written into the flat
gradient: split-K slabs reduce-added onto it), the MIOpen path for the rest,
and a whole ResNet-50 step with the convolutions bound to the flat buffers
against the unbound model."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from torch_distlearn_amd import _native

    _native.native()
    return torch.device("cuda", 0)


# (N, Cin, H, Cout): ResNet-50 bottleneck 1x1 shapes at small batch + M tails
SHAPES = [(4, 64, 56, 64), (4, 64, 56, 256), (4, 256, 56, 64), (2, 512, 28, 128), (2, 1024, 14, 256),
          (2, 2048, 7, 512), (3, 512, 7, 2048), (1, 128, 9, 512)]


@pytest.mark.parametrize("shape", SHAPES)
def test_conv1x1_matches_fp32(dev, shape):
    from torch_distlearn_amd.ops.conv import Conv1x1, ShadowBinding, conv1x1_supported

    N, cin, H, cout = shape
    g = torch.Generator(device=dev).manual_seed(cin * cout + H)
    cl = torch.channels_last
    x = torch.randn(N, cin, H, H, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w = torch.randn(cout, cin, 1, 1, device=dev, generator=g) * cin ** -0.5
    w16 = w.to(torch.bfloat16)
    go = torch.randn(N, cout, H, H, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    assert conv1x1_supported(x, cout)
    prior = torch.randn(cout, cin, device=dev, generator=g)
    g32 = prior.clone()  # the weight gradient is ADDED to what the flat gradient holds
    ready = []
    bind = ShadowBinding(w16.view(cout, cin), g32, lambda: ready.append(1))
    xi = x.detach().requires_grad_(True)
    wp = torch.nn.Parameter(w.clone())
    y = Conv1x1.apply(xi, wp, bind, None)
    y.backward(go)
    xr = x.float().detach().requires_grad_(True)
    wr = w16.float().detach().requires_grad_(True)
    yr = F.conv2d(xr, wr)
    yr.backward(go.float())
    torch.cuda.synchronize()
    assert y.is_contiguous(memory_format=cl) and y.dtype == torch.bfloat16
    assert _rel(y, yr) < 1e-2
    assert _rel(xi.grad, xr.grad) < 1e-2
    assert _rel(g32 - prior, wr.grad.view(cout, cin)) < 1e-3
    assert wp.grad is None and ready == [1]


@pytest.mark.parametrize("N,cin,H,cout", [(4, 256, 28, 128), (2, 64, 56, 256), (3, 512, 7, 2048)])
def test_conv1x1_bn_stats_epilogue(dev, N, cin, H, cout):
    """The forward epilogue's per-channel sum / sum of squares (deterministic
    partial rows + bn_rows_reduce: the input of the following BatchNorm)
    equal those of the stored bf16 output."""
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.ops.conv import Conv1x1, ShadowBinding

    C = _native.native()
    C.set_reduce_atomic(0)
    x = torch.randn(N, cin, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w16 = (torch.randn(cout, cin, device=dev) * 0.05).to(torch.bfloat16)
    stats = torch.zeros(2 * cout, device=dev)
    bind = ShadowBinding(w16, torch.zeros(cout, cin, device=dev), lambda: None)
    with torch.no_grad():
        y = Conv1x1.apply(x, torch.nn.Parameter(w16.float().view(cout, cin, 1, 1)), bind, stats)
    torch.cuda.synchronize()
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, cout)
    torch.testing.assert_close(stats[:cout], yf.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(stats[cout:], (yf * yf).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("k,stride,cin,cout,hw", [(3, 1, 64, 64, 28), (3, 2, 128, 128, 28), (1, 2, 256, 512, 28),
                                                  (7, 2, 3, 64, 64)])
def test_shadow_conv_matches_fp32(dev, k, stride, cin, cout, hw):
    from torch_distlearn_amd.ops.conv import ShadowBinding, ShadowConv

    g = torch.Generator(device=dev).manual_seed(k * 100 + cin)
    cl = torch.channels_last
    x = torch.randn(2, cin, hw, hw, device=dev, generator=g).to(torch.bfloat16).contiguous(memory_format=cl)
    w16 = (torch.randn(cout, cin, k, k, device=dev, generator=g) * (cin * k * k) ** -0.5).to(torch.bfloat16)
    g32 = torch.zeros(cout, cin, k, k, device=dev)
    bind = ShadowBinding(w16.view(-1), g32.view(-1), lambda: None)
    xi = x.detach().requires_grad_(True)
    y = ShadowConv.apply(xi, torch.nn.Parameter(w16.float()), bind, stride, k // 2)
    go = torch.randn_like(y)
    y.backward(go)
    xr, wr = x.float().detach().requires_grad_(True), w16.float().detach().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, k // 2)
    yr.backward(go.float())
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-2 and _rel(xi.grad, xr.grad) < 2e-2 and _rel(g32, wr.grad) < 2e-2


def test_resnet50_bound_convs_match_unbound(dev, monkeypatch):
    """One ResNet-50 training step (64x64 inputs, batch 8) with every
    convolution bound to the flat buffers (HIP 1x1 GEMMs + shadow MIOpen)
    against the same step with plain F.conv2d on cast weights: loss and the
    updated parameters agree to bf16 accuracy."""
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50, resnet

    tree = Tree(1, 1, host="127.0.0.1", port=29573, device=dev)
    x = torch.randn(8, 64, 64, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 100, (8,), device=dev)
    out = {}
    for bound in (True, False):
        model = ResNet50(num_classes=100, seed=0).to(dev)
        if not bound:
            model.attach_flat = None  # the trainer then leaves the convolutions unbound
        tr = DataParallelTrainer(model, tree, lr=0.05, backend="torch", compute_dtype=torch.bfloat16, max_batch=8)
        assert any(getattr(m, "bind", None) is not None for m in model.modules()) == bound
        tr.synchronize_parameters()
        before = tr.flat.data.clone()
        loss = float(tr.step(x, y))
        torch.cuda.synchronize()
        out[bound] = (loss, tr.flat.data - before)
    (lb, db), (lu, du) = out[True], out[False]
    assert abs(lb - lu) < 2e-2 * max(1.0, abs(lu))
    cos = float(F.cosine_similarity(db, du, dim=0))
    assert cos > 0.98, cos


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (2, 16, 9, 13), (3, 8, 7, 7)])
def test_maxpool_nhwc_matches_torch(dev, shape):
    """HIP channels-last 3x3/2 max pool (argmax bytes, gather backward) ==
    torch.nn.functional.max_pool2d forward and backward (same bf16 values,
    first-max tie rule)."""
    from torch_distlearn_amd.ops.pool import max_pool2d_nhwc

    N, C, H, W = shape
    g = torch.Generator(device=dev).manual_seed(C + H)
    # quantised values: plenty of ties inside the windows
    x = (torch.randn(N, C, H, W, device=dev, generator=g) * 2).round().div(2).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    xa = x.detach().requires_grad_(True)
    xb = x.detach().requires_grad_(True)
    ya = max_pool2d_nhwc(xa, 3, 2, 1)
    yb = F.max_pool2d(xb, 3, 2, 1)
    go = torch.randn_like(yb)
    ya.backward(go)
    yb.backward(go)
    torch.cuda.synchronize()
    assert torch.equal(ya, yb)
    torch.testing.assert_close(xa.grad.float(), xb.grad.float(), rtol=1e-2, atol=1e-2)


def test_weight_transposes_one_launch(dev):
    """ops.conv.WeightTransposes: many [Cout][Cin] shadows transposed by one
    transpose_many launch (ragged shapes, tails of the 64x64 tiles)."""
    from torch_distlearn_amd.ops.conv import ShadowBinding, WeightTransposes

    shapes = [(64, 64), (256, 64), (64, 256), (2048, 512), (96, 40), (8, 200)]
    ws = [torch.randn(co, ci, 1, 1, device=dev).to(torch.bfloat16) for co, ci in shapes]
    binds = [ShadowBinding(w, torch.zeros(w.shape, device=dev), lambda: None) for w in ws]
    wt = WeightTransposes(binds)
    wt.refresh()
    torch.cuda.synchronize()
    for w, b in zip(ws, binds):
        assert torch.equal(b.wt, w.view(w.shape[0], -1).t())
    ws[3].mul_(2)  # the shadow changes (optimizer step): the next refresh follows
    wt.refresh()
    torch.cuda.synchronize()
    assert torch.equal(binds[3].wt, ws[3].view(2048, 512).t())


def test_channels_last_weights_one_launch(dev):
    """ops.conv.ChannelsLastWeights: KxK shadows copied to channels-last by one
    weights_to_cl launch equal torch's own channels-last conversion."""
    from torch_distlearn_amd.ops.conv import ChannelsLastWeights, ShadowBinding

    shapes = [(64, 3, 7, 7), (64, 64, 3, 3), (512, 512, 3, 3), (24, 40, 3, 3)]
    ws = [torch.randn(s, device=dev).to(torch.bfloat16) for s in shapes]
    binds = [ShadowBinding(w, torch.zeros(w.shape, device=dev), lambda: None) for w in ws]
    cl = ChannelsLastWeights(binds, shapes)
    cl.refresh()
    torch.cuda.synchronize()
    for w, b in zip(ws, binds):
        assert b.wcl.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(b.wcl, w)


@pytest.mark.parametrize("N,cin,H,cout,padded", [(4, 64, 14, 64, False), (2, 128, 7, 256, True), (2, 64, 28, 128, True),
                                                 (3, 256, 9, 64, False), (2, 64, 16, 64, True)])
def test_conv3x3_matches_fp32(dev, N, cin, H, cout, padded):
    """ops.conv.Conv3x3 (streaming implicit-GEMM kernel, non-power-of-two H/W
    included) vs an fp32 conv2d: output, BN statistics, input gradient and the
    weight gradient reduce-added in [Cout][Cin][3][3] order; inputs either as
    zero-bordered interior views (what the BatchNorm kernels hand over) or
    plain channels-last tensors (padded copy inside)."""
    from torch_distlearn_amd.ops.bn_nhwc import padded_empty
    from torch_distlearn_amd.ops.conv import Conv3x3, ShadowBinding, conv3x3_supported

    g = torch.Generator(device=dev).manual_seed(N * cin + H)
    cl = torch.channels_last
    x0 = torch.randn(N, cin, H, H, device=dev, generator=g).to(torch.bfloat16)
    go0 = torch.randn(N, cout, H, H, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * (9 * cin) ** -0.5
    w16 = w.to(torch.bfloat16)
    if padded:
        x = padded_empty(N, cin, H, H, 1, dev)
        x.copy_(x0)
        go = padded_empty(N, cout, H, H, 1, dev)
        go.copy_(go0)
    else:
        x, go = x0.contiguous(memory_format=cl), go0.contiguous(memory_format=cl)
    assert conv3x3_supported(tuple(x.shape), cout)
    prior = torch.randn(cout, cin, 3, 3, device=dev, generator=g)
    g32 = prior.clone()
    ready = []
    bind = ShadowBinding(w16.view(-1), g32.view(-1), lambda: ready.append(1))
    bind.wcl = w16.contiguous(memory_format=cl)  # [Cout][3][3][Cin] in memory
    stats = torch.zeros(2 * cout, device=dev)
    xi = x.detach().requires_grad_(True)
    y = Conv3x3.apply(xi, torch.nn.Parameter(w.clone()), bind, stats)
    y.backward(go)
    xr = x0.float().requires_grad_(True)
    wr = w16.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, 1, 1)
    yr.backward(go0.float())
    torch.cuda.synchronize()
    assert _rel(y, yr) < 1e-2
    yf = y.float().permute(0, 2, 3, 1).reshape(-1, cout)
    torch.testing.assert_close(stats[:cout], yf.sum(0), rtol=1e-3, atol=1e-1)
    assert _rel(xi.grad, xr.grad) < 1e-2
    assert _rel(g32 - prior, wr.grad) < 1e-3 and ready == [1]


def test_bn_act_padded_output_and_dx(dev):
    """bn_act(out_pad=1, dx_pad=1): the output / input gradient are interior
    views of zero-bordered buffers with the same values as the plain path."""
    from torch_distlearn_amd.ops.bn_nhwc import bn_act

    N, C, H = 4, 128, 14
    x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w, b = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    go = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16)
    outs = []
    for pad in (0, 1):
        xi = x.detach().requires_grad_(True)
        seen = []
        xi.register_hook(seen.append)  # the gradient as handed over, before leaf accumulation
        y = bn_act(xi, w, b, None, None, relu=True, out_pad=pad, dx_pad=pad)
        y.backward(go)
        outs.append((y, seen[0]))
    torch.cuda.synchronize()
    (y0, d0), (y1, d1) = outs
    assert getattr(y1, "_dl_pad", 0) == 1 and getattr(d1, "_dl_pad", 0) == 1
    # (the BN reductions accumulate with atomics: bitwise equality is not promised)
    assert _rel(y1, y0) < 1e-2 and _rel(d1, d0) < 1e-2
    for t in (y1, d1):  # the border ring of the underlying [N][H+2][W+2][C] buffer is zero
        base = torch.as_strided(t, (N, H + 2, H + 2, C), ((H + 2) ** 2 * C, (H + 2) * C, C, 1),
                                t.storage_offset() - (H + 2 + 1) * C)
        ring = base.clone()
        ring[:, 1:-1, 1:-1, :] = 0
        assert float(ring.float().abs().max()) == 0.0


def test_bn_conv3x3_bn_chain_hands_over_padded(dev):
    """b1 -> Conv3x3 -> b2 as the bottleneck wires it: b1 writes its output
    zero-bordered, b2 its input gradient zero-bordered, and Conv3x3 uses both
    without a padding copy; the chain matches the same ops with plain
    tensors (pad copies inside Conv3x3)."""
    from torch_distlearn_amd.ops import conv as convmod
    from torch_distlearn_amd.ops.bn_nhwc import bn_act
    from torch_distlearn_amd.ops.conv import Conv3x3, ShadowBinding

    N, C, H = 4, 128, 14
    x = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w16 = (torch.randn(C, C, 3, 3, device=dev) * (9 * C) ** -0.5).to(torch.bfloat16)
    g1, b1 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    g2, b2 = torch.rand(C, device=dev) + 0.5, torch.randn(C, device=dev) * 0.1
    go = torch.randn(N, C, H, H, device=dev).to(torch.bfloat16)
    res = []
    for pad in (1, 0):
        g32 = torch.zeros(C, C, 3, 3, device=dev)
        bind = ShadowBinding(w16.view(-1), g32.view(-1), lambda: None)
        bind.wcl = w16.contiguous(memory_format=torch.channels_last)
        xi = x.detach().requires_grad_(True)
        before = convmod.PAD_COPIES[0]
        h = bn_act(xi, g1, b1, None, None, relu=True, out_pad=pad)
        h = Conv3x3.apply(h, torch.nn.Parameter(w16.float()), bind, None)
        h = bn_act(h, g2, b2, None, None, relu=True, dx_pad=pad)
        h.backward(go)
        torch.cuda.synchronize()
        res.append((h.detach().clone(), xi.grad.clone(), g32.clone(), convmod.PAD_COPIES[0] - before))
    (h1, d1, w1, copies1), (h0, d0, w0, copies0) = res
    assert copies1 == 0 and copies0 == 2
    assert _rel(h1, h0) < 1e-2 and _rel(d1, d0) < 2e-2 and _rel(w1, w0) < 1e-2
