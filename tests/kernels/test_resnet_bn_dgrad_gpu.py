"""ResNet-50 BatchNorm fusions across kernel boundaries: the masked residual
gradient added in the c1 dgrad epilogue, the hand-over between the two
branches of a block, the downsample BN applied on load by b3, the stem BN
applied on load by the max-pool, and the persistent zero-bordered buffers --
each against the unfused path and fp32 PyTorch.  (The BatchNorm backward sums
in the dgrad epilogue were removed in round 6, r5_resnet_bn_dgrad_ab.txt.)"""
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


@pytest.mark.parametrize("N,C,H,mid", [(4, 256, 14, 64), (2, 512, 7, 128)])
def test_masked_residual_gradient_in_c1_dgrad(dev, monkeypatch, N, C, H, mid):
    """Identity bottleneck form: x -> c1 (1x1) -> c3 (1x1) -> BN + residual(x) +
    ReLU.  With mask bits (relu mode 3) the BN's backward does not write the
    residual gradient: it hands (dy, mask bits) to c1, whose dgrad epilogue
    adds dy under the mask (conv_fwd_add with addend_mask).  x's gradient and
    every parameter gradient match the path that writes dres (to the noise of
    the BN reduce's fp32 atomics) and an fp32 PyTorch reference."""
    from torch_distlearn_amd.ops import bn_nhwc
    from torch_distlearn_amd.ops.conv import Conv1x1, ShadowBinding

    def run(masked):
        monkeypatch.setattr(bn_nhwc, "_MASKED_ADDEND", masked)
        g = torch.Generator(device=dev).manual_seed(8)
        mk = lambda *s: torch.randn(*s, device=dev, generator=g).to(BF).contiguous(memory_format=CL)  # noqa: E731
        x = mk(N, C, H, H).requires_grad_(True)
        w1 = (torch.randn(mid, C, 1, 1, device=dev, generator=g) * C ** -0.5).to(BF)
        w3 = (torch.randn(C, mid, 1, 1, device=dev, generator=g) * mid ** -0.5).to(BF)
        gamma = (torch.rand(C, device=dev, generator=g) + 0.5).requires_grad_(True)
        beta = (torch.randn(C, device=dev, generator=g) * 0.3).requires_grad_(True)
        go = mk(N, C, H, H)
        b1 = ShadowBinding(w1.reshape(mid, C), torch.zeros(mid, C, device=dev), lambda: None)
        b3 = ShadowBinding(w3.reshape(C, mid), torch.zeros(C, mid, device=dev), lambda: None)
        link = {}
        h = Conv1x1.apply(x, torch.nn.Parameter(w1.float()), b1, None, link, None)
        y3 = Conv1x1.apply(h, torch.nn.Parameter(w3.float()), b3, None, None, None)
        z = bn_nhwc.bn_act(y3, gamma, beta, None, None, residual=x, relu=True, acc=torch.zeros(4 * C, device=dev),
                           have_stats=False, res_sink=link)
        z.backward(go)
        torch.cuda.synchronize()
        assert ("gm" in link) is False and ("g" in link) is False  # consumed
        # fp32 reference of the same chain
        xr = x.detach().float().requires_grad_(True)
        gr, br = gamma.detach().clone().requires_grad_(True), beta.detach().clone().requires_grad_(True)
        hr = F.conv2d(xr, w1.float())
        zr = F.relu(F.batch_norm(F.conv2d(hr, w3.float()), None, None, gr, br, True, 0.1, 1e-5) + xr)
        zr.backward(go.float())
        return [x.grad, gamma.grad, beta.grad, b1.g32, b3.g32], [xr.grad, gr.grad, br.grad]

    on, ref = run(True)
    off, _ = run(False)
    for a, b in zip(on, off):
        assert _rel(a, b) < 1e-2
    for a, b in zip(on[:3], ref):
        assert _rel(a, b) < 3e-2


@pytest.mark.parametrize("branch", ["identity", "downsample_s2"])
def test_c1_backward_first_hand_over(dev, branch):
    """x feeds c1 (Conv1x1 with a residual link) and a second
    branch that hands its gradient of x to c1's dgrad (the identity residual's
    BatchNorm: res_sink; the stride-2 downsample conv: dx_sink).  Force c1's
    backward to run FIRST (separate backward calls): c1 marks the link done and
    the other branch must return its gradient through autograd -- x.grad
    equals the one joint backward where the hand-over happens."""
    from torch_distlearn_amd.ops.bn_nhwc import bn_act
    from torch_distlearn_amd.ops.conv import Conv1x1, Conv1x1S2, ShadowBinding

    N, C, H, mid = 4, 256, 14, 64

    def run(split):
        g = torch.Generator(device=dev).manual_seed(12)
        mk = lambda *s: torch.randn(*s, device=dev, generator=g).to(BF).contiguous(memory_format=CL)  # noqa: E731
        x = mk(N, C, H, H).requires_grad_(True)
        w1 = (torch.randn(mid, C, 1, 1, device=dev, generator=g) * C ** -0.5).to(BF)
        b1 = ShadowBinding(w1.reshape(mid, C), torch.zeros(mid, C, device=dev), lambda: None)
        link = {}
        a = Conv1x1.apply(x, torch.nn.Parameter(w1.float()), b1, None, link, None)
        if branch == "identity":
            y3 = mk(N, C, H, H).requires_grad_(True)
            gamma = torch.rand(C, device=dev, generator=g) + 0.5
            beta = torch.randn(C, device=dev, generator=g) * 0.3
            b = bn_act(y3, gamma, beta, None, None, residual=x, relu=True, acc=torch.zeros(4 * C, device=dev),
                       have_stats=False, res_sink=link)
        else:
            wd = (torch.randn(2 * C, C, 1, 1, device=dev, generator=g) * C ** -0.5).to(BF)
            bd = ShadowBinding(wd.reshape(2 * C, C), torch.zeros(2 * C, C, device=dev), lambda: None)
            bd.wt = None
            b = Conv1x1S2.apply(x, torch.nn.Parameter(wd.float()), bd, None, link)
        ga, gb = mk(*a.shape), mk(*b.shape)
        if split:  # c1's backward first, then the other branch's
            a.backward(ga, retain_graph=True)
            b.backward(gb)
        else:
            torch.autograd.backward([b, a], [gb, ga])
        torch.cuda.synchronize()
        return x.grad.float(), link

    joint, _ = run(False)
    first, link = run(True)
    assert link.get("done")
    assert _rel(first, joint) < 1e-2


@pytest.mark.parametrize("N,C,H", [(4, 256, 14), (2, 512, 7)])
def test_deferred_residual_bn_apply(dev, N, C, H):
    """The downsample branch's BN (no ReLU) deferred into the BN + residual +
    ReLU that consumes it (bn_act defer_apply; csrc bn_nhwc.hip ResBn) and its
    backward fused into that BN's backward (ResBnBwd: the residual BN's sums
    ride the reduce pass, its input gradient is written where g was): the
    block output and the running statistics are BITWISE those of the path that
    runs the downsample BN on its own (statistics given), every gradient equal
    to the noise of the backward sums' fp32 atomics, and materialize() runs
    the deferred apply for another consumer."""
    from torch_distlearn_amd.ops.bn_nhwc import bn_act, materialize

    def run(defer):
        g = torch.Generator(device=dev).manual_seed(17)
        mk = lambda *s: torch.randn(*s, device=dev, generator=g).to(BF).contiguous(memory_format=CL)  # noqa: E731
        y3, yd = mk(N, C, H, H).requires_grad_(True), mk(N, C, H, H).requires_grad_(True)
        p = [(torch.rand(C, device=dev, generator=g) + 0.5).requires_grad_(True) for _ in range(2)]
        q = [(torch.randn(C, device=dev, generator=g) * 0.3).requires_grad_(True) for _ in range(2)]
        rs = [(torch.zeros(C, device=dev), torch.ones(C, device=dev)) for _ in range(2)]

        def acc_of(t):
            tf = t.detach().float().permute(0, 2, 3, 1).reshape(-1, C)
            return torch.cat([tf.sum(0), (tf * tf).sum(0), torch.zeros(2 * C, device=dev)])

        s = bn_act(yd, p[1], q[1], *rs[1], relu=False, acc=acc_of(yd), have_stats=True, defer_apply=defer)
        if defer:
            assert getattr(s, "_dl_res_bn", None) is not None
        z = bn_act(y3, p[0], q[0], *rs[0], residual=s, relu=True, acc=acc_of(y3), have_stats=True)
        go = mk(N, C, H, H)
        z.backward(go)
        torch.cuda.synchronize()
        return [z, y3.grad, yd.grad, p[0].grad, p[1].grad, q[0].grad, q[1].grad, *rs[0], *rs[1]]

    a, b = run(False), run(True)
    for i in (0, 7, 8, 9, 10):  # output, running statistics
        assert torch.equal(a[i], b[i]), i
    for i in range(1, 7):  # input and parameter gradients
        assert _rel(b[i], a[i]) < 1e-3, (i, _rel(b[i], a[i]))
    # materialize(): the deferred output written as the plain apply writes it
    g = torch.Generator(device=dev).manual_seed(3)
    yd = torch.randn(N, C, H, H, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    w, bb = torch.rand(C, device=dev, generator=g) + 0.5, torch.randn(C, device=dev, generator=g)
    tf = yd.float().permute(0, 2, 3, 1).reshape(-1, C)
    acc = torch.cat([tf.sum(0), (tf * tf).sum(0), torch.zeros(2 * C, device=dev)])
    with torch.no_grad():
        ref = bn_act(yd, w, bb, None, None, relu=False, acc=acc.clone(), have_stats=True)
        d = bn_act(yd, w, bb, None, None, relu=False, acc=acc.clone(), have_stats=True, defer_apply=True)
        materialize(d)
    torch.cuda.synchronize()
    assert torch.equal(ref, d)


def test_resnet50_step_deferred_down_bn(dev, monkeypatch):
    """The whole ResNet-50 step with the downsample BNs applied on load by the
    blocks' b3 against the separate apply: same loss and gradients (to the
    run-to-run noise of the fp32 statistics atomics)."""
    from torch_distlearn_amd import FlatParams
    from torch_distlearn_amd.models import ResNet50
    from torch_distlearn_amd.models import resnet as R

    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(16, 3, 64, 64, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    y = torch.randint(0, 1000, (16,), device=dev, generator=g)
    out = []
    for on in (False, True):
        monkeypatch.setattr(R, "_DEFER_DOWN_BN", on)
        model = ResNet50(num_classes=1000, seed=0).to(dev)
        flat = FlatParams(model, grads=True, shadow_bf16=True)
        model.attach_flat(flat)
        flat.grad.zero_()
        loss, _ = model.forward_loss(x, y, BF)
        loss.backward()
        torch.cuda.synchronize()
        rm = torch.cat([blk.down[1].running_mean for blk in model.blocks if blk.down is not None])
        out.append((float(loss), flat.grad.clone(), rm))
    assert abs(out[0][0] - out[1][0]) < 1e-6
    assert _rel(out[1][1], out[0][1]) < 2e-2
    assert _rel(out[1][2], out[0][2]) < 1e-5


@pytest.mark.parametrize("N,C,H", [(4, 64, 56), (2, 64, 112)])
def test_stem_pool_applies_bn_on_load(dev, N, C, H):
    """The stem BN + ReLU applied by the 3x3/2 max-pool on load (bn_act
    defer_pool; csrc pool_nhwc.hip PoolBn): pooled output, argmax choice and
    the BN's running statistics BITWISE those of the BN apply + pool path,
    gradients to the noise of the backward sums' fp32 atomics."""
    from torch_distlearn_amd.ops.bn_nhwc import bn_act
    from torch_distlearn_amd.ops.pool import max_pool2d_nhwc

    def run(defer):
        g = torch.Generator(device=dev).manual_seed(23)
        x = torch.randn(N, C, H, H, device=dev, generator=g).to(BF).contiguous(memory_format=CL).requires_grad_(True)
        w = (torch.rand(C, device=dev, generator=g) + 0.5).requires_grad_(True)
        b = (torch.randn(C, device=dev, generator=g) * 0.3).requires_grad_(True)
        rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        tf = x.detach().float().permute(0, 2, 3, 1).reshape(-1, C)
        acc = torch.cat([tf.sum(0), (tf * tf).sum(0), torch.zeros(2 * C, device=dev)])
        z = bn_act(x, w, b, rm, rv, relu=True, acc=acc, have_stats=True, defer_pool=defer)
        assert (getattr(z, "_dl_pool_bn", None) is not None) == defer
        p = max_pool2d_nhwc(z, 3, 2, 1)
        go = torch.randn(p.shape, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
        p.backward(go)
        torch.cuda.synchronize()
        return [p, rm, rv], [x.grad, w.grad, b.grad]

    (ea, ga), (eb, gb) = run(False), run(True)
    for u, v in zip(ea, eb):
        assert torch.equal(u, v)
    for u, v in zip(ga, gb):
        assert _rel(v, u) < 1e-3


def test_resnet50_step_deferred_stem_bn(dev, monkeypatch):
    """The whole ResNet-50 step with the stem BN applied by the max-pool on load
    against the separate apply: same loss, gradients to atomics noise."""
    from torch_distlearn_amd import FlatParams
    from torch_distlearn_amd.models import ResNet50
    from torch_distlearn_amd.models import resnet as R

    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(16, 3, 64, 64, device=dev, generator=g).to(BF).contiguous(memory_format=CL)
    y = torch.randint(0, 1000, (16,), device=dev, generator=g)
    out = []
    for on in (False, True):
        monkeypatch.setattr(R, "_DEFER_STEM_BN", on)
        model = ResNet50(num_classes=1000, seed=0).to(dev)
        flat = FlatParams(model, grads=True, shadow_bf16=True)
        model.attach_flat(flat)
        flat.grad.zero_()
        loss, _ = model.forward_loss(x, y, BF)
        loss.backward()
        torch.cuda.synchronize()
        out.append((float(loss), flat.grad.clone(), model.stem_bn.running_var.clone()))
    assert abs(out[0][0] - out[1][0]) < 1e-6
    assert _rel(out[1][1], out[0][1]) < 2e-2
    assert torch.equal(out[1][2], out[0][2])


def test_persistent_pad_buffers_reused_and_guarded(dev, monkeypatch):
    """Persistent zero-bordered BN buffers (ops/bn_nhwc.py padded_buffer): a
    training step releases every view, so the next step reuses the same memory;
    a second forward while the first one's views are still saved gets buffers
    of its own, so the first forward's backward is unaffected."""
    from torch_distlearn_amd import FlatParams
    from torch_distlearn_amd.models import ResNet50
    from torch_distlearn_amd.models import resnet as R

    monkeypatch.setattr(R, "_PAD_PERSIST", True)
    g = torch.Generator(device=dev).manual_seed(8)
    xs = [torch.randn(8, 3, 64, 64, device=dev, generator=g).to(BF).contiguous(memory_format=CL) for _ in range(2)]
    ys = [torch.randint(0, 1000, (8,), device=dev, generator=g) for _ in range(2)]
    model = ResNet50(num_classes=1000, seed=0).to(dev)
    flat = FlatParams(model, grads=True, shadow_bf16=True)
    model.attach_flat(flat)
    caches = [m.pad_bufs for m in model.modules() if hasattr(m, "pad_bufs")]

    def bases():
        return {(id(c), k): e[0].data_ptr() for c in caches for k, e in c.items()}

    grads = []
    for i in range(2):
        flat.grad.zero_()
        loss, _ = model.forward_loss(xs[i], ys[i], BF)
        loss.backward()
        torch.cuda.synchronize()
        grads.append(flat.grad.clone())
        if i == 0:
            first = bases()
    assert first, "no persistent pad buffers were used"
    assert all(e[1]() is None for c in caches for e in c.values()), "a pad-buffer view outlived its step"
    assert bases() == first
    # two forwards, then the first one's backward: the second forward must not
    # overwrite the views the first saved (the flat gradient is overwritten per
    # backward, not accumulated, so only one backward runs)
    flat.grad.zero_()
    l0, _ = model.forward_loss(xs[0], ys[0], BF)
    l1, _ = model.forward_loss(xs[1], ys[1], BF)
    l0.backward()
    torch.cuda.synchronize()
    assert _rel(flat.grad, grads[0]) < 2e-2
    del l1
