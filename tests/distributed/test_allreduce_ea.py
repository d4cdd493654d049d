"""AllReduceEA oracle (port of test/test_AllReduceEA.lua:4-43).

tau=3, alpha=0.4, 5 epochs of random 45-53 steps per node; parameters wander
with an amplitude that halves every step, ``averageParameters`` every step,
``synchronizeCenter`` at epoch end.  Oracle: max-abs difference of the
parameters across nodes < 1e-6.  Also checks the centers are bit-identical
(scattered) and that a stale (out-of-place replaced) parameter table is
handled (SURVEY §3.5 hazard).
"""
import random

import pytest
import torch

from tests import mp


def _ea_worker(rank, world, port, trials, replace_out_of_place):
    from torch_distlearn_amd import AllReduceEA, Tree

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    outs = []
    for trial in range(trials):
        rng = random.Random(77 * trial + rank)
        torch.manual_seed(1 + rank + 31 * trial)
        ea = AllReduceEA(tree, 3, 0.4)
        params = [torch.randn(7)]
        ea.synchronizeParameters(params)
        slowit = 1.0
        rounds = 0
        for _epoch in range(5):
            steps = rng.randint(45, 53)
            for _ in range(steps):
                if replace_out_of_place:
                    params[0] = params[0] + torch.randn(7) / slowit  # new tensor object every step
                else:
                    params[0].add_(torch.randn(7) / slowit)
                rounds += ea.averageParameters(params)
                slowit *= 2
            ea.synchronizeCenter(params)
        outs.append((params[0].clone(), ea.center[64:71].clone(), rounds))
    tree.comm.barrier()
    return outs


@pytest.mark.parametrize("world", [2, 4, 8])
def test_allreduce_ea_converges(world):
    res = mp.run(_ea_worker, world, 10, False)  # 10 trials: test/test_AllReduceEA.lua:23
    for trial in range(10):
        p0, c0, _ = res[0][trial]
        for r in range(1, world):
            p, c, _ = res[r][trial]
            assert abs(p0 - p).max() < 1e-6, f"params of node {r+1} too far: {abs(p0-p).max()}"
            assert c0.tobytes() == c.tobytes(), "centers must be bit-identical after synchronizeCenter"


def test_allreduce_ea_out_of_place_params():
    res = mp.run(_ea_worker, 2, 1, True)
    p0, _, n0 = res[0][0]
    p1, _, _ = res[1][0]
    assert n0 > 0
    assert abs(p0 - p1).max() < 1e-6


def _idle_worker(rank, world, port, active):
    from torch_distlearn_amd import AllReduceEA, Tree

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    ea = AllReduceEA(tree, 2, 0.3)
    torch.manual_seed(5 + rank)
    params = [torch.randn(9)]
    ea.synchronizeParameters(params)
    for _ in range(active[rank]):
        params[0].add_(torch.randn(9))
        ea.averageParameters(params)
    ea.synchronizeCenter(params)
    first = params[0].clone()
    ea.synchronizeCenter(params)  # every node idle: the drain must not move anything (AllReduceEA.lua:52)
    return first, params[0].clone(), ea.center[64:73].clone()


@pytest.mark.parametrize("active", [(0, 0), (3, 5), (0, 4)])
def test_allreduce_ea_idle_drain_leaves_params(active):
    """A second synchronizeCenter in a row (every node at step 0) leaves the
    params untouched, like the reference's ``if step > 0`` guard; a mix of
    idle and active nodes (a deadlock in the reference) completes."""
    res = mp.run(_idle_worker, 2, list(active))
    for first, second, _ in res:
        assert first.tobytes() == second.tobytes()
    assert res[0][2].tobytes() == res[1][2].tobytes()
