"""The reference MNIST convnet's fused one-kernel training step
(csrc/kernels/mnist.hip, models/mnist_hip.py) against an fp32 PyTorch
reference of the same model: loss, log-probabilities and every parameter
gradient; and the trainer on the HIP executor against the torch backend."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from torch_distlearn_amd import _native

    _native.native()
    return torch.device("cuda", 0)


@pytest.mark.parametrize("B,dtype", [(1, torch.float32), (1, torch.bfloat16), (5, torch.float32), (16, torch.bfloat16)])
def test_mnist_step_matches_fp32(dev, B, dtype):
    from torch_distlearn_amd import FlatParams
    from torch_distlearn_amd.models import MnistConvNet
    from torch_distlearn_amd.models.mnist_hip import MnistHIPExecutor

    g = torch.Generator(device=dev).manual_seed(B)
    x = torch.randn(B, 32, 32, 1, device=dev, generator=g).to(dtype)
    y = torch.randint(0, 10, (B,), device=dev, generator=g)
    ref = MnistConvNet(seed=1).to(dev)
    lp_ref = ref(x.float())
    L = ref.loss(lp_ref, y)
    L.backward()
    m = MnistConvNet(seed=1).to(dev)
    flat = FlatParams(m, grads=True)
    ex = MnistHIPExecutor(m, flat, max_batch=16)
    flat.grad.zero_()
    loss = ex.forward_backward(x, y)
    torch.cuda.synchronize()
    torch.testing.assert_close(loss, L.detach(), rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ex.last_logits(), lp_ref.detach(), rtol=1e-4, atol=1e-4)
    for (n, pr), gv in zip(ref.named_parameters(), flat.views_of(flat.grad)):
        torch.testing.assert_close(gv, pr.grad, rtol=1e-3, atol=1e-5, msg=n)
    lp = ex.predict(x)
    torch.testing.assert_close(lp, lp_ref.detach(), rtol=1e-4, atol=1e-4)


def test_mnist_trainer_hip_vs_torch(dev):
    """Graph-captured trainer steps on the fused kernel track the PyTorch path."""
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import MnistConvNet

    tree = Tree(1, 1, host="127.0.0.1", port=29591, device=dev)
    g = torch.Generator(device=dev).manual_seed(3)
    xs = torch.randn(20, 4, 1024, device=dev, generator=g)
    ys = torch.randint(0, 10, (20, 4), device=dev, generator=g)
    res = {}
    for backend, graph in (("hip", True), ("torch", False)):
        m = MnistConvNet(seed=0).to(dev)
        tr = DataParallelTrainer(m, tree, lr=0.05, backend=backend, compute_dtype=torch.float32, graph=graph,
                                 max_batch=4)
        tr.synchronize_parameters()
        losses = [float(tr.step(xs[i], ys[i])) for i in range(20)]
        # the public predict (the trainer passes batch_stats to every
        # executor; the MNIST net has no BatchNorm, so both modes agree)
        lps = [tr.predict(xs[0], batch_stats=bs) for bs in (False, True)]
        res[backend] = (losses, tr.flat.data.clone(), lps)
    (lh, ph, lph), (lt, pt, lpt) = res["hip"], res["torch"]
    assert max(abs(a - b) for a, b in zip(lh, lt)) < 1e-3
    assert float((ph - pt).abs().max()) < 1e-4
    assert torch.equal(lph[0], lph[1])
    torch.testing.assert_close(lph[0], lpt[0], rtol=1e-3, atol=1e-3)
