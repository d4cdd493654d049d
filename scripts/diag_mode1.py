"""Mode-1 (atomic reductions) determinism / graph-vs-eager diagnostic: per-step
losses and final parameter differences for eager/graph runs in both modes."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(mode, graph, port):
    os.environ["DISTLEARN_REDUCE_ATOMIC"] = str(mode)
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet

    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=port, device=dev)
    model = CifarConvNet(seed=7).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.02, backend="hip", compute_dtype=torch.bfloat16, graph=graph,
                             max_batch=32)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(0)
    xs = torch.randn(4, 32, 32, 32, 3, device=dev, generator=g).to(torch.bfloat16)
    ys = torch.randint(0, 10, (4, 32), device=dev, generator=g)
    losses = [float(tr.step(xs[i], ys[i])) for i in range(4)]
    torch.cuda.synchronize()
    return losses, tr.flat.data.clone()


if __name__ == "__main__":
    res = {}
    for key in [(0, False), (0, True), (1, False), (1, False), (1, True), (1, True)]:
        l, p = run(*key, port=29800)
        tag = f"mode{key[0]}-{'graph' if key[1] else 'eager'}"
        ref = res.setdefault(tag, (l, p))
        print(tag, " ".join(f"{v:.5f}" for v in l), "dp_vs_first_same_tag", float((p - ref[1]).abs().max()), flush=True)
        res.setdefault("all", []).append((tag, l, p))
    base = res["all"][0]
    for tag, l, p in res["all"]:
        print(tag, "max|dloss| vs mode0-eager", max(abs(a - b) for a, b in zip(l, base[1])),
              "max|dp|", float((p - base[2]).abs().max()))
