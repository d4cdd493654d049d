#!/usr/bin/env python3
"""Which Python call sites launch the elementwise copy / fill / add kernels of a
ResNet-50 training step (torch.profiler with stacks, one eager step at batch 32)."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50

    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29597, device=dev)
    B = 32
    x = torch.randn(B, 224, 224, 3, device=dev).to(torch.bfloat16)
    y = torch.randint(0, 1000, (B,), device=dev)
    tr = DataParallelTrainer(ResNet50(seed=0).to(dev), tree, lr=0.02, backend="torch", compute_dtype=torch.bfloat16,
                             graph=False, max_batch=B)
    tr.synchronize_parameters()
    for _ in range(2):
        tr.step(x, y)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile

    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        tr.step(x, y)
        torch.cuda.synchronize()
    sites = Counter()
    for ev in prof.events():
        if ev.name in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::clone",
                       "aten::contiguous", "aten::to", "aten::_to_copy"):
            st = [f for f in (ev.stack or []) if "torch_distlearn_amd" in f or "bench" in f]
            sites[(ev.name, st[0] if st else "?", str(ev.input_shapes)[:80])] += 1
    for (name, site, shp), n in sites.most_common(40):
        print(f"{n:4d}  {name:16s} {site}  {shp}")


if __name__ == "__main__":
    main()
