"""Multi-rank rehearsal of the GPU training path on ONE MI355X: 2 ranks share
cuda:0 (RCCL refuses two ranks on one GPU -- "Duplicate GPU detected" -- so
the data plane here is torch's gloo backend on device tensors), running the
hand-written HIP executor, the gradient bucketer, the participation slot,
the uneven-step drain and the epoch-end winner broadcast; parameters must be
BITWISE identical across ranks (the reference's AllReduceSGD oracle,
test/test_AllReduceSGD.lua:37-39).  The RCCL + hipGraph data plane itself is
exercised at world 1 by the other GPU tests; with one rank per GPU over RCCL
by tests/kernels/test_rccl_multigpu.py (its ``rccl`` rows need >= 2 GPUs and
skip on a 1-GPU box) and by ``bench.py --gpus N``."""
import pytest
import torch

from tests import mp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, uneven, algo):
    import torch

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tree = Tree(rank + 1, world, host="127.0.0.1", port=port, device=dev, backend="gloo")
    model = CifarConvNet(seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.05, algo=algo, tau=2, alpha=0.3, backend="hip",
                             compute_dtype=torch.bfloat16, bucket_bytes=1 << 20, graph=False, max_batch=16)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    steps = 4 + (2 * rank if uneven else 0)
    for _ in range(steps):
        x = torch.randn(16, 32, 32, 3, device=dev, generator=g).to(torch.bfloat16)
        y = torch.randint(0, 10, (16,), device=dev, generator=g)
        tr.step(x, y)
    tr.synchronize()
    torch.cuda.synchronize()
    return {"p": tr.flat.data.float().cpu(), "nb": len(tr.bucketer.ranges) if tr.bucketer else 0,
            "finite": bool(torch.isfinite(tr.flat.data).all())}


@pytest.fixture(scope="module")
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("uneven", [False, True])
def test_two_ranks_sgd_bitwise(_gpu, uneven):
    res = mp.run(_worker, 2, uneven, "sgd")
    assert res[0]["nb"] == 3, "CIFAR net with 1 MiB buckets: 3 buckets overlap the backward"
    assert all(r["finite"] for r in res)
    assert (res[0]["p"] == res[1]["p"]).all()


def test_two_ranks_ea_runs(_gpu):
    res = mp.run(_worker, 2, True, "ea")
    assert all(r["finite"] for r in res)
