"""Which aten ops of one eager ResNet-50 training step copy memory, and from
where (the step's rocprofv3 trace shows ~89 __amd_rocclr_copyBuffer per step):
every aten op under a TorchDispatchMode is logged with the innermost repo
frame that issued it; copy-like ops are summed by (op, frame).

    python scripts/diag_r50_copies.py [--batch 64]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COPY_OPS = ("copy_", "clone", "_to_copy", "contiguous", "cat", "stack", "index", "masked_fill", "add", "zero_",
            "fill_", "zeros", "new_zeros", "where", "to")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__ if hasattr(func, "__name__") else str(func)
        if any(name.split(".")[0].startswith(c) for c in COPY_OPS):
            frame = "?"
            for fr in reversed(traceback.extract_stack()[:-1]):
                if fr.filename.startswith(ROOT) and "diag_r50_copies" not in fr.filename:
                    frame = f"{os.path.relpath(fr.filename, ROOT)}:{fr.lineno} {fr.name}"
                    break
            self.ops[(name, frame)] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    a = ap.parse_args()
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50
    from torch_distlearn_amd.utils.color_print import set_verbose

    set_verbose(False)
    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29531, device=dev)
    model = ResNet50(seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.02, backend="torch", compute_dtype=torch.bfloat16, graph=False,
                             max_batch=a.batch)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(a.batch, 224, 224, 3, device=dev, generator=g).to(torch.bfloat16)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)
    tr.step(x, y)  # warm-up (allocations, transposed shadows)
    torch.cuda.synchronize()
    log = Log()
    with log:
        tr.step(x, y)
    torch.cuda.synchronize()
    print(f"# copy-like aten ops of one eager ResNet-50 step (batch {a.batch}), by issuing repo frame")
    for (op, fr), n in sorted(log.ops.items(), key=lambda kv: -kv[1]):
        print(f"{n:5d}  {op:40s} {fr}")


if __name__ == "__main__":
    main()
