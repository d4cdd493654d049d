"""Generalised-geometry MFMA convolutions (csrc/kernels/conv_igemm.hip
conv_fwd_ex / conv_wgrad_ex) against fp32 PyTorch: stride-2 3x3 and 1x1
convolutions (the ResNet-50 downsampling convs), non-square kernels, the
epilogue output map (phase-interleaved stores, in-place accumulate) and the
weight gradients with a separate dy geometry."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module")
def C():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from torch_distlearn_amd import _native

    return _native.native()


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _tile_fwd(cout):
    return 0 if cout % 128 == 0 else 2


def _tile_wgrad(cout):
    return 2 if cout % 128 == 0 else 1


# (N, Hi, Cin, Cout, K, stride, pad)
FWD_SHAPES = [(4, 14, 64, 64, 3, 2, 1), (2, 28, 128, 128, 3, 2, 1), (3, 8, 64, 128, 1, 2, 0), (2, 14, 256, 512, 1, 2, 0),
              (2, 10, 64, 64, 3, 1, 1), (2, 7, 64, 128, 3, 2, 1)]


@pytest.mark.parametrize("shape", FWD_SHAPES)
@pytest.mark.parametrize("splits", [1, 2])
def test_conv_fwd_ex_strided(C, shape, splits):
    N, Hi, cin, cout, k, S, p = shape
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(hash(shape) % 1000)
    x = torch.randn(N, Hi, Hi, cin, device=dev, generator=g).to(BF)
    w = (torch.randn(cout, k, k, cin, device=dev, generator=g) * (1.0 / (k * k * cin)) ** 0.5).to(BF)
    Ho = (Hi + 2 * p - k) // S + 1
    xp = F.pad(x, (0, 0, p, p, p, p)).contiguous()
    y = torch.empty(N, Ho, Ho, cout, device=dev, dtype=BF)
    slab = torch.empty(splits * N * Ho * Ho * cout, device=dev) if splits > 1 else None
    C.conv_fwd_ex(xp.data_ptr(), w.data_ptr(), y.data_ptr(), 0, 0 if slab is None else slab.data_ptr(), N, Ho, Ho,
                  Hi + 2 * p, Hi + 2 * p, cin, cout, k, k, S, 0, 0, 0, 0, 0, 0, _tile_fwd(cout), splits,
                  torch.cuda.current_stream().cuda_stream)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), stride=S, padding=p)
    torch.cuda.synchronize()
    assert _rel(y.permute(0, 3, 1, 2), ref) < 1e-2


def test_conv_fwd_ex_stats(C):
    """BN statistics rows from the epilogue of a strided conv."""
    N, Hi, cin, cout = 4, 14, 64, 128
    dev = torch.device("cuda")
    x = torch.randn(N, Hi + 2, Hi + 2, cin, device=dev).to(BF)
    x[:, 0] = 0
    x[:, -1] = 0
    x[:, :, 0] = 0
    x[:, :, -1] = 0
    w = (torch.randn(cout, 3, 3, cin, device=dev) * 0.05).to(BF)
    Ho = 7
    y = torch.empty(N, Ho, Ho, cout, device=dev, dtype=BF)
    rows = torch.zeros(64, 2, cout, device=dev)
    T = C.conv_fwd_ex(x.data_ptr(), w.data_ptr(), y.data_ptr(), rows.data_ptr(), 0, N, Ho, Ho, Hi + 2, Hi + 2, cin,
                      cout, 3, 3, 2, 0, 0, 0, 0, 0, 0, 0, 1, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    yf = y.float().reshape(-1, cout)
    assert T == (N * Ho * Ho + 127) // 128
    torch.testing.assert_close(rows[:T, 0].sum(0), yf.sum(0), rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(rows[:T, 1].sum(0), (yf * yf).sum(0), rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("kh,kw,cin", [(2, 1, 64), (1, 2, 128), (2, 2, 64), (4, 4, 64), (4, 4, 16)])
def test_conv_fwd_ex_nonsquare_with_output_map(C, kh, kw, cin):
    """A KH x KW 'valid' conv over a buffer, stored through the output map at
    rows (2*oh + 1, 2*ow) of a larger tensor, accumulated onto what is there
    (cin 16: the per-lane tap path of the stem's space-to-depth conv)."""
    N, Ho, cout = 3, 6, 64
    dev = torch.device("cuda")
    Hp, Wp = Ho + kh - 1, Ho + kw - 1
    xb = torch.randn(N, Hp, Wp, cin, device=dev).to(BF)
    w = (torch.randn(cout, kh, kw, cin, device=dev) * 0.05).to(BF)
    Hf = 2 * Ho + 1
    full = torch.randn(N, Hf, Hf, cout, device=dev).to(BF)
    before = full.clone()
    C.conv_fwd_ex(xb.data_ptr(), w.data_ptr(), full.data_ptr(), 0, 0, N, Ho, Ho, Hp, Wp, cin, cout, kh, kw, 1, 2, 1, 0,
                  Hf, Hf * Hf, full.data_ptr(), 2, 1, torch.cuda.current_stream().cuda_stream)
    ref = F.conv2d(xb.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float())  # [N, cout, Ho, Ho]
    torch.cuda.synchronize()
    want = before.float().clone()
    want[:, 1::2, 0:2 * Ho:2, :] += ref.permute(0, 2, 3, 1)
    assert _rel(full[:, 1::2, 0:2 * Ho:2], want[:, 1::2, 0:2 * Ho:2]) < 1e-2
    untouched = torch.ones(N, Hf, Hf, dtype=torch.bool, device=dev)
    untouched[:, 1::2, 0:2 * Ho:2] = False
    assert torch.equal(full[untouched], before[untouched])


# (N, Hi, Cin, Cout, K, stride, pad, dy interior pad)
WG_SHAPES = [(4, 14, 64, 64, 3, 2, 1, 0), (2, 28, 128, 128, 3, 2, 1, 1), (3, 8, 64, 128, 1, 2, 0, 0),
             (2, 14, 256, 256, 1, 2, 0, 0), (2, 7, 64, 128, 3, 2, 1, 0)]


@pytest.mark.parametrize("shape", WG_SHAPES)
@pytest.mark.parametrize("splits", [1, 3])
def test_conv_wgrad_ex_strided(C, shape, splits):
    N, Hi, cin, cout, k, S, p, dp = shape
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(N, Hi, Hi, cin, device=dev, generator=g).to(BF)
    Ho = (Hi + 2 * p - k) // S + 1
    dy = torch.randn(N, Ho, Ho, cout, device=dev, generator=g).to(BF)
    xp = F.pad(x, (0, 0, p, p, p, p)).contiguous()
    dyp = F.pad(dy, (0, 0, dp, dp, dp, dp)).contiguous()
    K = k * k * cin
    out = torch.empty(splits, cout, K, device=dev)
    C.conv_wgrad_ex(dyp.data_ptr(), xp.data_ptr(), out.data_ptr(), N, Ho, Ho, Hi + 2 * p, Hi + 2 * p, Ho + 2 * dp,
                    Ho + 2 * dp, dp, cin, cout, k, k, S, splits, K, _tile_wgrad(cout),
                    torch.cuda.current_stream().cuda_stream)
    xr = x.permute(0, 3, 1, 2).float().requires_grad_(False)
    wr = torch.zeros(cout, cin, k, k, device=dev, requires_grad=True)
    yr = F.conv2d(xr, wr, stride=S, padding=p)
    yr.backward(dy.permute(0, 3, 1, 2).float())
    ref = wr.grad.permute(0, 2, 3, 1).reshape(cout, K)  # [Cout][kh][kw][Cin]
    torch.cuda.synchronize()
    assert _rel(out.sum(0), ref) < 1e-2
