"""Micro-benchmark of the per-step prep kernel parts (gather+normalise+pad,
layer-1 weight pack, dgrad weight flip-transposes) and the small per-step
kernels of the CIFAR executor; graph-replayed, GPU time per launch."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import _native
from torch_distlearn_amd.data import DeviceLoader, PartitionedDataset
from torch_distlearn_amd.models import CifarConvNet, make_executor
from torch_distlearn_amd.ops.flat import FlatParams


def timeit(fn, iters=100):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / iters


def main():
    dev = torch.device("cuda")
    C = _native.native()
    model = CifarConvNet(seed=0).to(dev)
    flat = FlatParams(model, grads=True, shadow_bf16=True)
    ex = make_executor(model, flat, max_batch=128)
    g = torch.Generator(device=dev).manual_seed(0)
    imgs = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labs = torch.randint(0, 10, (50000,), device=dev, generator=g)
    ld = DeviceLoader(PartitionedDataset(imgs, labs, device=dev), "permutation", 128, seed=0)
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    x = torch.randn(128, 32, 32, 3, device=dev).to(torch.bfloat16)
    print(f"empty-ish (fill 1 elem)   {timeit(lambda: C.fill_f32(flat.grad.data_ptr(), 0.0, 4, -1, 0.0, s())):7.2f} us")
    print(f"prep gather+pack+transp  {timeit(lambda: ex._prep(ld, s(), with_transposes=True)):7.2f} us")
    print(f"prep gather+pack         {timeit(lambda: ex._prep(ld, s(), with_transposes=False)):7.2f} us")
    print(f"prep tensor+pack+transp  {timeit(lambda: ex._prep(x, s(), with_transposes=True)):7.2f} us")
    print(f"prep tensor+pack         {timeit(lambda: ex._prep(x, s(), with_transposes=False)):7.2f} us")
    print(f"transposes only          {timeit(lambda: ex._prep_transposes(s())):7.2f} us")


def small_kernels():
    """Isolated small per-step kernels of the executor (graph-replayed)."""
    dev = torch.device("cuda")
    C = _native.native()
    s = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    for T, Cc, M in ((1024, 64, 131072), (256, 128, 32768), (384, 256, 8192), (400, 512, 2048)):
        part = torch.randn(T, 2, Cc, device=dev).abs()
        gam = torch.ones(Cc, device=dev)
        bet = torch.zeros(Cc, device=dev)
        rm = torch.zeros(Cc, device=dev)
        rv = torch.ones(Cc, device=dev)
        coef = torch.empty(4, Cc, device=dev)
        acoef = torch.empty(3, Cc, device=dev)
        dg = torch.empty(Cc, device=dev)
        t1 = timeit(lambda: C.bn_finalize(part.data_ptr(), T, Cc, M, gam.data_ptr(), bet.data_ptr(), 0, rm.data_ptr(),
                                          rv.data_ptr(), 1e-3, 0.1, 0, coef.data_ptr(), s()))
        t2 = timeit(lambda: C.bn_bwd_finalize(part.data_ptr(), T, Cc, M, gam.data_ptr(), coef.data_ptr(), dg.data_ptr(),
                                              dg.data_ptr(), acoef.data_ptr(), s()))
        print(f"bn_finalize T={T:5d} C={Cc:4d}: {t1:6.2f} us   bn_bwd_finalize: {t2:6.2f} us")


if __name__ == "__main__":
    main()
    small_kernels()
