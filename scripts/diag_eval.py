"""Bisect the HIP executor's held-out accuracy against torch on the same
trained weights.  Prints one line per probe."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torch_distlearn_amd import LocalhostTree  # noqa: E402
from torch_distlearn_amd.data import Dataset, DeviceLoader  # noqa: E402
from torch_distlearn_amd.engine import DataParallelTrainer  # noqa: E402
from torch_distlearn_amd.models import CifarConvNet  # noqa: E402


@torch.no_grad()
def acc_of(fn, batcher, n):
    batcher.reset()
    ok = tot = 0
    for _ in range(n):
        x, y = batcher.getBatch()
        p = fn(x)
        ok += int((p.argmax(1) == y).sum())
        tot += y.numel()
    return ok / tot


def main():
    B = int(os.environ.get("B", "32"))
    steps = int(os.environ.get("STEPS", "64"))
    mode = os.environ.get("PATHMODE", "fast")
    dev = torch.device("cuda")
    tree = LocalhostTree(1, 1, port=29811, device=dev)
    train = Dataset("cifar10", 1, 1, train=True, synthetic_size=int(os.environ.get("NTRAIN", "2048")), device=dev)
    test = Dataset("cifar10", 1, 1, train=False, synthetic_size=int(os.environ.get("NTEST", "512")), device=dev)
    chunk = int(os.environ.get("CHUNK", "0"))
    torch.manual_seed(0)
    model = CifarConvNet(seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.1, backend="hip", compute_dtype=torch.bfloat16,
                             graph=mode != "eager", max_batch=B)
    tr.synchronize_parameters()
    if mode == "eager" or mode == "graph1":
        tb = train.sampledBatcher("label-uniform", B, dtype=torch.bfloat16, seed=1)
        for _ in range(steps):
            x, y = tb.getBatch()
            loss = tr.step(x, y)
    else:
        dl = DeviceLoader(train, "label-uniform", B, seed=1)
        tr.prepare(dl, 16)
        if chunk:
            tb_ = test.sampledBatcher("linear", B, dtype=torch.bfloat16)
            done = 0
            while done < steps:
                loss = tr.run(dl, min(chunk, steps - done), unroll=16)
                done += min(chunk, steps - done)
                model.eval()
                a_hip = acc_of(tr.predict, tb_, tb_.numBatches())
                a_t = acc_of(lambda x: model(x, compute_dtype=torch.float32), tb_, tb_.numBatches())
                model.train()
                print(f"  step {done}: loss {float(loss):.5f} hip-test {a_hip:.4f} torch-eval-test {a_t:.4f}", flush=True)
        else:
            loss = tr.run(dl, steps, unroll=16)
    torch.cuda.synchronize()
    print(f"mode={mode} B={B} steps={steps} loss={float(loss):.5f} red={os.environ.get('DISTLEARN_REDUCE_ATOMIC', '2')}")
    tr.synchronize()
    test_b = test.sampledBatcher("linear", B, dtype=torch.bfloat16)
    trl_b = train.sampledBatcher("linear", B, dtype=torch.bfloat16)
    nt = test_b.numBatches()
    print(f"  hip predict  test {acc_of(tr.predict, test_b, nt):.4f}  train {acc_of(tr.predict, trl_b, 8):.4f}")
    model.eval()
    f32 = lambda x: model(x, compute_dtype=torch.float32)  # noqa: E731
    print(f"  torch eval   test {acc_of(f32, test_b, nt):.4f}  train {acc_of(f32, trl_b, 8):.4f}")
    saved = [b.clone() for b in model.buffers()]
    model.train()
    print(f"  torch train  test {acc_of(f32, test_b, nt):.4f}  train {acc_of(f32, trl_b, 8):.4f}")
    for b, v in zip(model.buffers(), saved):
        b.copy_(v)
    model.eval()
    # running stats vs the batch statistics of a training batch (torch fp32 forward hooks)
    x, _ = trl_b.getBatch()
    torch.set_grad_enabled(False)
    h = x.permute(0, 3, 1, 2).float()
    import torch.nn.functional as F
    for i in range(model.nblocks):
        w, b, g, beta, rm, rv = model.block_params(i)
        h = F.conv2d(h, w.permute(0, 3, 1, 2), b, padding=2)
        bm = h.mean((0, 2, 3))
        bv = h.var((0, 2, 3))
        print(f"  blk{i}: rm err {float((rm - bm).norm() / bm.norm()):.3e}  rv err {float((rv - bv).norm() / bv.norm()):.3e}"
              f"  |bm| {float(bm.abs().mean()):.3e} bv {float(bv.mean()):.3e} rv {float(rv.mean()):.3e}")
        h = F.batch_norm(h, None, None, g, beta, True, 0.1, model.bn_eps)
        h = F.max_pool2d(F.relu(h), 2, 2)
    # HIP predict vs torch eval logits on one test batch
    test_b.reset()
    x, y = test_b.getBatch()
    a, r = tr.predict(x), f32(x)
    print(f"  predict vs torch eval rel {float((a - r).norm() / r.norm()):.3e}")


if __name__ == "__main__":
    main()
