"""AllReduceSGD oracle (port of test/test_AllReduceSGD.lua:4-42, not of its code).

World sizes {2,4,8} on gloo over 127.0.0.1, random 4-13 steps per node per
epoch (uneven -> exercises the drain protocol), 5 epochs, grads = 1/steps.
Oracle: parameters BITWISE identical on every node after
``synchronizeParameters``.  Run for a plain tensor table, for a FlatParams
(zero-copy path) and for the bucketed overlap path.
"""
import random

import pytest
import torch

from tests import mp


def _sgd_worker(rank, world, port, trials, mode):
    from torch_distlearn_amd import AllReduceSGD, FlatParams, Tree
    from torch_distlearn_amd.parallel import GradBucketer

    tree = Tree(rank + 1, world, base=2, host="127.0.0.1", port=port)
    outs = []
    for trial in range(trials):
        rng = random.Random(1000 * trial + rank)
        torch.manual_seed(rank + 17 * trial)
        if mode == "table":
            params = [torch.randn(7)]
            grads = [torch.zeros(7)]
            sgd = AllReduceSGD(tree)
            sgd.synchronizeParameters(params)
            for _epoch in range(5):
                steps = rng.randint(4, 13)
                for _ in range(steps):
                    grads[0].fill_(1.0 / steps)
                    sgd.sumAndNormalizeGradients(grads)
                    params[0].add_(grads[0])
                sgd.synchronizeParameters(params)
            outs.append(params[0].clone())
        else:
            # two "layers" so the flat buffer has several tensors / buckets
            w = torch.nn.Parameter(torch.randn(7, 3))
            b = torch.nn.Parameter(torch.randn(5))
            flat = FlatParams([w, b])
            bucketer = GradBucketer(tree.comm, flat, bucket_bytes=64, hooks=False,
                                    wire="bf16" if mode.startswith("bucket16") else "fp32") \
                if mode.startswith("bucket") else None
            if mode.startswith("bucket16"):
                assert bucketer.wire16 and flat.grad16 is not None
            sgd = AllReduceSGD(tree, bucketer=bucketer)
            if mode.endswith("_early"):  # per-bucket update right after each all-reduce
                assert sgd.enable_bucket_updates(flat, lambda: -1.0)
                assert bucketer.nb > 1 and bucketer.hdr_first
            sgd.synchronizeParameters(flat)
            for _epoch in range(5):
                steps = rng.randint(4, 13)
                for _ in range(steps):
                    flat.zero_grad()
                    w.grad.fill_(1.0 / steps)
                    b.grad.fill_(-0.5 / steps)
                    if bucketer is not None:
                        for k in range(bucketer.nb):
                            bucketer.mark_bucket_ready(k)
                    sgd.step(flat, lr=-1.0)  # p -= -1 * g/n  == p += g/n (reference adds grads)
                    if mode.endswith("_early"):
                        assert bucketer.early_applied
                sgd.synchronizeParameters(flat)
            outs.append(torch.cat([w.detach().reshape(-1), b.detach().reshape(-1)]).clone())
    tree.comm.barrier()
    return outs


TRIALS = 10


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode", ["table", "flat", "bucket", "bucket16", "bucket_early"])
def test_allreduce_sgd_bitwise(world, mode):
    # 10 randomized trials like test/test_AllReduceSGD.lua:23
    res = mp.run(_sgd_worker, world, TRIALS, mode)
    for trial in range(TRIALS):
        r0 = res[0][trial]
        for r in range(1, world):
            assert (r0 == res[r][trial]).all() and r0.tobytes() == res[r][trial].tobytes(), f"node {r+1} params differ (trial {trial}, mode {mode})"


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bf16_wire_matches_fp32_wire(world):
    """grad_comm_dtype bf16 (bf16 bucket all-reduce, fp32 participation count)
    ends at the fp32-wire parameters to bf16 tolerance, with uneven epochs
    (drain + winner broadcast), on 2, 4 and 8 gloo ranks (the wire's sum is
    accumulated in bf16 per hop: the bound has to hold at the largest world)."""
    r32 = mp.run(_sgd_worker, world, 3, "bucket")
    r16 = mp.run(_sgd_worker, world, 3, "bucket16")
    for t in range(3):
        a, b = r32[0][t], r16[0][t]
        assert abs(a - b).max() <= 2e-2 * max(1.0, abs(a).max()), (a, b)


@pytest.mark.parametrize("wire", ["bucket", "bucket16"])
def test_bucket_updates_match_single_update(wire):
    """Per-bucket SGD on the comm stream right after each all-reduce
    (participation count all-reduced with the first bucket; draining nodes
    issue the same collectives and update nothing) ends at the single
    full-buffer update, uneven epochs on 4 gloo ranks.  Not bitwise: the
    header bucket's all-reduce no longer carries the header, and gloo's ring
    sums an element in an order set by its chunk of the message (replicas
    stay bitwise equal: test_allreduce_sgd_bitwise[bucket_early])."""
    a = mp.run(_sgd_worker, 4, 3, wire)
    b = mp.run(_sgd_worker, 4, 3, wire + "_early")
    tol = 1e-6 if wire == "bucket" else 2e-2
    for r in range(4):
        for t in range(3):
            x, y = a[r][t], b[r][t]
            assert abs(x - y).max() <= tol * max(1.0, abs(x).max()), (r, t, abs(x - y).max())
