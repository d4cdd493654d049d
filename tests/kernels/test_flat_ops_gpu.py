"""HIP flat-bucket kernels (csrc/kernels/flat_ops.hip) vs fp32 PyTorch
references: K3 scale-by-count, K4 fill+slot, K5 fused SGD (+momentum, wd,
bf16 shadow), K8/K10 elastic step (+pending), K9 add, cast.  Sizes include
non-multiple-of-block tails (all multiples of 4: FlatParams pads to 64)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [4, 68, 4096 + 12, 4_328_972]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from torch_distlearn_amd import _native

    _native.native()
    return torch.device("cuda:0")


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("mom", [False, True])
@pytest.mark.parametrize("count", [1.0, 3.0])
def test_sgd_update(dev, n, mom, count):
    from torch_distlearn_amd.ops.flat import sgd_update_

    g0 = torch.Generator(device=dev).manual_seed(n)
    p = torch.randn(n, device=dev, generator=g0)
    g = torch.randn(n, device=dev, generator=g0)
    m = torch.randn(n, device=dev, generator=g0) if mom else None
    slot = torch.tensor([count], device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    lr, mu, wd = 0.1, 0.9, 1e-4
    # reference
    d = g * (1.0 / count if count > 1 else 1.0) + wd * p
    mref = None
    if mom:
        mref = mu * m + d
        d = mref
    pref = p - lr * d
    sgd_update_(p, g, lr, slot=slot, mom=m, momentum=mu, weight_decay=wd, shadow=sh)
    torch.cuda.synchronize()
    torch.testing.assert_close(p, pref, rtol=1e-6, atol=1e-6)
    if mom:
        torch.testing.assert_close(m, mref, rtol=1e-6, atol=1e-6)
    assert torch.equal(sh, p.to(torch.bfloat16))


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("pending", [False, True])
def test_elastic_step(dev, n, pending):
    from torch_distlearn_amd.ops.flat import elastic_step_

    g0 = torch.Generator(device=dev).manual_seed(7 + n)
    p = torch.randn(n, device=dev, generator=g0)
    c = torch.randn(n, device=dev, generator=g0)
    pend = torch.randn(n, device=dev, generator=g0) if pending else None
    out = torch.empty(n, device=dev)
    alpha = 0.2
    cref = c + pend if pending else c.clone()
    dref = alpha * (p - cref)
    pref = p - dref
    elastic_step_(p, c, out, alpha, pending=pend)
    torch.cuda.synchronize()
    torch.testing.assert_close(c, cref, rtol=0, atol=0)
    torch.testing.assert_close(out, dref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(p, pref, rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("n", SIZES)
def test_elastic_step_wire16(dev, n):
    """AsyncEA bf16 delta wire kernel vs the fp32 reference: the wire copy is
    bf16(alpha (p - c)) (round to nearest even, like torch), the fp32 delta is
    exactly that bf16 value, p moved by exactly it, shadow = bf16(p)."""
    from torch_distlearn_amd.ops.flat import elastic_step_wire16_

    g0 = torch.Generator(device=dev).manual_seed(11 + n)
    p = torch.randn(n, device=dev, generator=g0)
    c = torch.randn(n, device=dev, generator=g0)
    p0, c0 = p.clone(), c.clone()
    out = torch.empty(n, device=dev)
    out16 = torch.empty(n, dtype=torch.bfloat16, device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    elastic_step_wire16_(p, c, out, out16, 0.2, shadow=sh)
    torch.cuda.synchronize()
    d16 = (0.2 * (p0 - c0)).to(torch.bfloat16)
    assert torch.equal(out16, d16)
    assert torch.equal(out, d16.float())
    assert torch.equal(p, p0 - d16.float())
    assert torch.equal(c, c0)
    assert torch.equal(sh, p.to(torch.bfloat16))


@pytest.mark.parametrize("n", SIZES)
def test_fill_scale_add(dev, n):
    from torch_distlearn_amd.ops.flat import add_, fill_, scale_by_count_

    x = torch.randn(n, device=dev)
    fill_(x, 0.0, slot_value=1.0, slot_index=0)
    ref = torch.zeros(n, device=dev)
    ref[0] = 1.0
    assert torch.equal(x, ref)
    y = torch.randn(n, device=dev)
    yref = y.clone()
    scale_by_count_(y, torch.tensor([4.0], device=dev))
    torch.testing.assert_close(y, yref / 4.0, rtol=1e-6, atol=0)
    z = torch.randn(n, device=dev)
    zref = z + y
    add_(z, y)
    torch.testing.assert_close(z, zref, rtol=0, atol=0)


def test_rccl_world1_identity(dev):
    """world_size=1 RCCL communicator: collectives are the identity and the
    participation slot round-trips."""
    import os

    from torch_distlearn_amd import FlatParams, Tree

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    tree = Tree(1, 1, host="127.0.0.1", port=29611, device=dev)
    m = torch.nn.Linear(33, 7).to(dev)
    f = FlatParams(m)
    f.grad.normal_()
    f.grad[0] = 1.0
    before = f.grad.clone()
    from torch_distlearn_amd.parallel.tree import FlatBuffer

    _, n = tree.allReduce(FlatBuffer(f.grad))
    torch.cuda.synchronize()
    assert int(n.item()) == 1
    assert torch.equal(f.grad, before)
    t = torch.randn(1000, device=dev)
    t0 = t.clone()
    tree.scatter([t])
    torch.cuda.synchronize()
    assert torch.equal(t, t0)


def test_sum_and_normalize_slot_in_buffer(dev):
    """sumAndNormalizeGradients on a FlatParams whose all-reduced slot says
    n = 4, with a buffer spanning thousands of workgroups: every element is
    divided (the slot itself lives in the buffer's header and is read, never
    scaled).  Regression for the slot/scale race."""
    from torch_distlearn_amd import FlatParams
    from torch_distlearn_amd.ops.flat import HEADER, scale_by_count_

    m = torch.nn.Sequential(torch.nn.Linear(1024, 2048), torch.nn.Linear(2048, 1000)).to(dev)
    f = FlatParams(m)
    f.grad.normal_()
    f.grad[0] = 4.0
    ref = f.grad.clone()
    scale_by_count_(f.grad[HEADER:], f.slot)
    torch.cuda.synchronize()
    assert float(f.grad[0]) == 4.0
    torch.testing.assert_close(f.grad[HEADER:], ref[HEADER:] / 4.0, rtol=1e-6, atol=0)
    with pytest.raises(ValueError):
        scale_by_count_(f.grad, f.slot)
