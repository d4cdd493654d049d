"""Step time of the 1-GPU CIFAR-10 training step while R CUs are held by
workgroups with RCCL's all-reduce footprint (256 threads, ~288 registers per
wave, 19.7 KiB LDS: csrc/testing/diag.hip).  On a multi-GPU run the bucketed
all-reduce overlaps the backward pass on a comm stream; compute kernels whose
workgroups do not fit beside an RCCL workgroup lose those CUs.  This measures
that effect on one GPU (R = 0 is the plain step).

    python scripts/emulate_rccl.py [--cus 0,16,32,64] [--steps 400]

A negative count -R launches R light one-wave workgroups instead (no LDS, few
registers: they fit beside anything), the control for the cost of a second
active queue alone.
"""

def _native_testing():
    from torch_distlearn_amd import _native

    return _native.testing()

import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from torch_distlearn_amd import Tree
from torch_distlearn_amd._native import native
from torch_distlearn_amd.data import DeviceLoader, PartitionedDataset
from torch_distlearn_amd.engine import DataParallelTrainer
from torch_distlearn_amd.models import CifarConvNet

ap = argparse.ArgumentParser()
ap.add_argument("--cus", default="0,16,32,64")
ap.add_argument("--steps", type=int, default=400)
ap.add_argument("--port", type=int, default=29731)
a = ap.parse_args()
dev = torch.device("cuda", 0)
C = native()
tree = Tree(1, 1, host="127.0.0.1", port=a.port, device=dev)
model = CifarConvNet(seed=0).to(dev)
tr = DataParallelTrainer(model, tree, lr=0.1, backend="hip", compute_dtype=torch.bfloat16, bucket_bytes=1 << 20,
                         graph=True, max_batch=128)
tr.synchronize_parameters()
g = torch.Generator(device=dev).manual_seed(1234)
imgs = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
labs = torch.randint(0, 10, (50000,), device=dev, generator=g)
loader = DeviceLoader(PartitionedDataset(imgs, labs, device=dev), "permutation", 128, seed=0)
tr.run(loader, 24)
torch.cuda.synchronize()
side = torch.cuda.Stream(device=dev)
sink = torch.zeros(1024, device=dev)
for r in [int(v) for v in a.cus.split(",")]:
    torch.cuda.synchronize()
    # hold the CUs for longer than the timed run (~0.5 ms/step bound)
    _native_testing().occupy_cus(r, int(a.steps * 600 + 20000), sink.data_ptr(), side.cuda_stream)
    torch.cuda._sleep(2_000_000)  # let the occupying workgroups land first
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tr.run(loader, a.steps)
    e1.record()
    torch.cuda.synchronize()
    print(f"occupied CUs {r:3d}{' (light)' if r < 0 else ''}: {e0.elapsed_time(e1) / a.steps * 1e3:7.1f} us/step", flush=True)
tr.finish()
