"""ResNet-50 hipGraph vs eager, root cause check: from the
SAME initial state and batch, one training step eager and one step replayed
from a captured graph; compare the loss, every gradient (flat buffer) and the
updated parameters with each other AND with an fp32 PyTorch reference step.
If graph-vs-eager differences are of the size of the bf16-vs-fp32 error, the
graph path is as correct as eager (bf16 algorithm-selection numerics)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def main():
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import ResNet50

    dev = torch.device("cuda", 0)
    tree = Tree(1, 1, host="127.0.0.1", port=29595, device=dev)
    B = int(os.environ.get("DIAG_BATCH", "32"))
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, 224, 224, 3, device=dev, generator=g).to(torch.bfloat16)
    y = torch.randint(0, 1000, (B,), device=dev, generator=g)
    out = {}
    for mode in ("eager", "graph", "eager2"):
        model = ResNet50(seed=0).to(dev)
        tr = DataParallelTrainer(model, tree, lr=0.02, backend="torch", compute_dtype=torch.bfloat16,
                                 graph=mode == "graph", max_batch=B)
        tr.synchronize_parameters()
        p0 = tr.flat.data.clone()
        loss = float(tr.step(x, y))
        torch.cuda.synchronize()
        out[mode] = (loss, tr.flat.grad.clone(), tr.flat.data - p0,
                     [b.clone() for b in model.buffers()])
    # fp32 reference: same init, same batch, plain autograd
    ref = ResNet50(seed=0).to(dev)
    logp = ref(x.float(), compute_dtype=torch.float32)
    L = ref.loss(logp, y)
    L.backward()
    from torch_distlearn_amd import FlatParams

    fr = FlatParams(ref, grads=False)
    gref = torch.zeros_like(out["eager"][1])
    for t, o, n in zip(fr.leaves, fr.offsets, fr.numels):
        gref[o:o + n] = t.grad.reshape(-1)
    le, ge, de, be = out["eager"]
    lg, gg, dg, bg = out["graph"]
    l2, g2, d2, b2 = out["eager2"]
    H = 64
    print(f"loss eager {le:.6f} graph {lg:.6f} eager2 {l2:.6f} fp32 {float(L):.6f}")
    print(f"grad rel: graph-vs-eager {rel(gg[H:], ge[H:]):.3e}  eager2-vs-eager {rel(g2[H:], ge[H:]):.3e}  "
          f"eager-vs-fp32 {rel(ge[H:], gref[H:]):.3e}  graph-vs-fp32 {rel(gg[H:], gref[H:]):.3e}")
    print(f"update rel: graph-vs-eager {rel(dg, de):.3e}  eager2-vs-eager {rel(d2, de):.3e}")
    print("buffers (running stats) max rel graph-vs-eager", max(rel(a, b) for a, b in zip(bg, be)))


if __name__ == "__main__":
    main()
