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


def test_resnet50_graph_matches_eager():
    """VERDICT r1 item 3b as a test (scripts/diag_r50_graph.py at test size):
    from the same state and batch, one step eager and one replayed from a
    captured hipGraph agree on the loss, and their gradients are as close to
    an fp32 autograd reference as each other (the only graph-vs-eager
    difference allowed is bf16 algorithm-selection noise)."""
    import os

    from torch_distlearn_amd import FlatParams, Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29573, device=dev)
    B = 8
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, 64, 64, 3, device=dev, generator=g).to(torch.bfloat16)
    y = torch.randint(0, 100, (B,), device=dev, generator=g)
    out = {}
    for mode in ("eager", "graph"):
        model = ResNet50(num_classes=100, seed=0).to(dev)
        tr = DataParallelTrainer(model, tree, lr=0.02, backend="torch", compute_dtype=torch.bfloat16,
                                 graph=mode == "graph", max_batch=B)
        tr.synchronize_parameters()
        p0 = tr.flat.data.clone()
        loss = float(tr.step(x, y))
        torch.cuda.synchronize()
        out[mode] = (loss, tr.flat.grad.clone(), tr.flat.data - p0)
        if mode == "graph":
            assert tr.captures >= 1
        tr.finish()
    ref = ResNet50(num_classes=100, seed=0).to(dev)
    L = ref.loss(ref(x.float(), compute_dtype=torch.float32), y)
    L.backward()
    fr = FlatParams(ref, grads=False)
    gref = torch.zeros_like(out["eager"][1])
    for t, o, n in zip(fr.leaves, fr.offsets, fr.numels):
        gref[o:o + n] = t.grad.reshape(-1)
    H = 64
    (le, ge, de), (lg, gg, dg) = out["eager"], out["graph"]

    def rel(a, b):
        return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))

    lr32 = float(L.detach())
    assert abs(lg - le) < 1e-2 * abs(le) and abs(le - lr32) < 2e-2 * abs(lr32), (le, lg, lr32)
    e_ref, g_ref = rel(ge[H:], gref[H:]), rel(gg[H:], gref[H:])
    assert e_ref < 0.1 and g_ref < 1.5 * e_ref + 1e-3, (e_ref, g_ref)
    assert rel(dg, de) < 0.1


@pytest.mark.parametrize("c,hw,relu,res", [(64, 28, True, False), (256, 14, True, True), (128, 7, False, False),
                                           (2048, 7, True, True), (512, 7, False, True)])
def test_bn_act_hip_matches_fp32(c, hw, relu, res):
    """ops.bn_nhwc.bn_act (HIP) vs an fp32 PyTorch reference of
    act(BN(x) [+ r]): output, dx, dweight, dbias, dres, running stats."""
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.ops.bn_nhwc import bn_act

    _native.native()
    torch.manual_seed(c + hw)
    dev = "cuda"
    n = 16
    cl = torch.channels_last
    xb = (torch.randn(n, c, hw, hw, device=dev) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    rb = torch.randn(n, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl) if res else None
    w, b = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.2
    go = torch.randn(n, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)

    def run(hip):
        x = (xb if hip else xb.float()).detach().requires_grad_(True)
        r = None if rb is None else (rb if hip else rb.float()).detach().requires_grad_(True)
        wi, bi = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        rm, rv = torch.zeros(c, device=dev), torch.ones(c, device=dev)
        if hip:
            y = bn_act(x, wi, bi, rm, rv, r, relu)
        else:
            y = F.batch_norm(x, rm, rv, wi, bi, True, 0.1, 1e-5)
            y = y + r if r is not None else y
            y = F.relu(y) if relu else y
        y.backward(go.to(y.dtype))
        outs = [y, x.grad, wi.grad, bi.grad, rm, rv] + ([r.grad] if r is not None else [])
        return [o.float() for o in outs]

    got, ref = run(True), run(False)
    names = ["y", "dx", "dw", "db", "running_mean", "running_var", "dres"]
    for name, a, r in zip(names, got, ref):
        rel = float((a - r).norm() / (r.norm() + 1e-12))
        assert rel < 2e-2, (name, rel)


@pytest.mark.parametrize("c,hw", [(256, 14), (2048, 7), (64, 56)])
def test_bn_residual_mask_bits_bitwise(c, hw, monkeypatch):
    """BN + residual + ReLU: the backward's ReLU mask from the forward's mask
    bits (relu mode 3, 1/16 of y's bytes, y not kept) is exactly the mask of
    the output y -- the residual gradient (the masked dy) equals
    where(y > 0, dy, 0) bit for bit -- and mode 3 agrees with mode 1 (mask
    read from y) to the run-to-run noise of the statistics' fp32 atomics."""
    from torch_distlearn_amd import _native
    from torch_distlearn_amd.ops import bn_nhwc

    _native.native()
    torch.manual_seed(c)
    dev, n, cl = "cuda", 8, torch.channels_last
    xb = (torch.randn(n, c, hw, hw, device=dev) * 2 + 0.3).to(torch.bfloat16).contiguous(memory_format=cl)
    rb = torch.randn(n, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w, b = torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev) * 0.2
    go = torch.randn(n, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    outs = []
    for bits in (False, True):
        monkeypatch.setattr(bn_nhwc, "_MASK_BITS", bits)
        x, r = xb.detach().requires_grad_(True), rb.detach().requires_grad_(True)
        wi, bi = w.clone().requires_grad_(True), b.clone().requires_grad_(True)
        y = bn_nhwc.bn_act(x, wi, bi, torch.zeros(c, device=dev), torch.ones(c, device=dev), r, True)
        assert y.grad_fn.__class__.__name__ == "_BnActBackward"
        y.backward(go)
        torch.cuda.synchronize()
        outs.append([y, x.grad, r.grad, wi.grad, bi.grad])
    (y0, dx0, dr0, dw0, db0), (y1, dx1, dr1, dw1, db1) = outs
    assert torch.equal(dr1, torch.where(y1 > 0, go, torch.zeros_like(go)))  # mode 3: bits == y's mask
    assert torch.equal(dr0, torch.where(y0 > 0, go, torch.zeros_like(go)))
    for a, b_ in ((y0, y1), (dx0, dx1), (dw0, dw1), (db0, db1), (dr0, dr1)):
        assert float((a.float() - b_.float()).norm() / (b_.float().norm() + 1e-12)) < 1e-2


def test_resnet50_mixed_bn_train_step(monkeypatch):
    # the MIOpen BN path (DISTLEARN_RESNET_BN=mixed); the default is the HIP BN
    from torch_distlearn_amd.models import resnet

    monkeypatch.setattr(resnet, "_BN_MODE", "mixed")
    test_resnet50_train_step()


@pytest.mark.parametrize("N,H,W,C,p", [(3, 56, 56, 64, 1), (2, 7, 5, 512, 1), (2, 6, 9, 16, 2)])
def test_zero_border_only_touches_the_border(N, H, W, C, p):
    """zero_border_nhwc enumerates the border pixels directly (bn_nhwc.hip):
    the ring is zeroed, the interior is left as it was."""
    from torch_distlearn_amd import _native
    from torch_distlearn_amd._native import stream_handle

    buf = torch.randn(N, H + 2 * p, W + 2 * p, C, device="cuda").to(torch.bfloat16) + 5
    before = buf.clone()
    _native.native().zero_border_nhwc(buf.data_ptr(), N, H, W, C, p, stream_handle())
    torch.cuda.synchronize()
    inner = (slice(None), slice(p, p + H), slice(p, p + W))
    assert torch.equal(buf[inner], before[inner])
    ring = torch.ones(H + 2 * p, W + 2 * p, dtype=torch.bool, device="cuda")
    ring[p:p + H, p:p + W] = False
    assert (buf[:, ring] == 0).all()


def test_resnet50_eval_bn_on_hip_kernel(monkeypatch):
    """ResNet-50 eval / predict runs its BatchNorms on the
    same HIP apply kernel as training, from the running statistics (no fp32
    copy, no F.batch_norm), after a few training steps: log-probabilities match
    the F.batch_norm eval path (fp32 BN on the same bf16 activations) and the
    predicted classes agree."""
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50
    from torch_distlearn_amd.models import resnet as R

    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29581, device=dev)
    model = ResNet50(num_classes=100, seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.02, backend="torch", compute_dtype=torch.bfloat16, max_batch=32)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(3)
    xs = torch.randn(4, 32, 64, 64, 3, device=dev, generator=g).to(torch.bfloat16)
    ys = torch.randint(0, 100, (4, 32), device=dev, generator=g)
    for k in range(3):
        tr.step(xs[k], ys[k])
    torch.cuda.synchronize()
    calls = []
    orig = R._BN.act

    def spy(self, x, *a, **kw):
        calls.append(self.hip_eval_ok(x, kw.get("residual")))
        return orig(self, x, *a, **kw)

    monkeypatch.setattr(R._BN, "act", spy)
    lp_hip = tr.predict(xs[3]).float()
    assert calls and all(calls), "eval BatchNorms did not take the HIP kernel"
    monkeypatch.setattr(R, "_BN_EVAL_HIP", False)
    lp_ref = tr.predict(xs[3]).float()
    torch.cuda.synchronize()
    rel = float((lp_hip - lp_ref).norm() / lp_ref.norm())
    assert rel < 2e-2, rel
    assert float((lp_hip.argmax(1) == lp_ref.argmax(1)).float().mean()) >= 0.9

