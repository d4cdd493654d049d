"""World > 1 overlap-policy selection (engine.py select_policy /
agree_on_policy) on gloo: every rank measures its own
step time per candidate policy; a step is as slow as its slowest rank, so the
ranks agree on the policy whose MAXIMUM is smallest -- the same one on every
rank even when the local minima disagree."""
import pytest

from tests import mp

# rank -> local ms per policy: rank 0 alone would pick "full", rank 1 "reserve";
# max over ranks: full 0.50, reserve 0.41 -> "reserve"
TIMES = [{"full": 0.30, "reserve": 0.40}, {"full": 0.50, "reserve": 0.41}, {"full": 0.35, "reserve": 0.38},
         {"full": 0.31, "reserve": 0.39}]


class _FakeExecutor:
    def __init__(self):
        self.calls = []

    def policies(self):
        return {"full": {"dgrad_stages": 3, "cu_reserve": 0}, "reserve": {"dgrad_stages": 2, "cu_reserve": 32}}

    def set_policy(self, dgrad_stages, cu_reserve):
        self.calls.append((dgrad_stages, cu_reserve))


def _worker(rank, world, port):
    import torch

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer, agree_on_policy

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    name, table = agree_on_policy(tree.comm, TIMES[rank])
    tr = DataParallelTrainer(torch.nn.Linear(4, 2), tree, lr=0.1)
    ex = _FakeExecutor()
    tr.executor, tr.graph = ex, True
    seen = []

    def fake_time(loader, reps):
        seen.append(ex.calls[-1])
        return TIMES[rank]["full" if ex.calls[-1][0] == 3 else "reserve"]

    tr._time_step_graph = fake_time
    pol = tr.select_policy(None)
    again = tr.select_policy(None)  # runs once
    return {"agree": (name, table), "policy": pol, "again": again is pol, "calls": ex.calls, "seen": seen}


@pytest.mark.parametrize("world", [2, 4])
def test_ranks_agree_on_the_fastest_slowest_rank(world):
    res = mp.run(_worker, world)
    want_table = {p: max(TIMES[r][p] for r in range(world)) for p in ("full", "reserve")}
    want = min(want_table, key=want_table.get)
    assert want == "reserve"
    for r in res:
        name, table = r["agree"]
        assert name == want and table == pytest.approx(want_table)
        pol = r["policy"]
        assert pol["chosen"] == want and pol["ms_per_step"] == pytest.approx(want_table)
        assert r["again"]
        # both candidates measured (sorted order), then the winner set for good
        assert r["seen"] == [(3, 0), (2, 32), (2, 32), (3, 0)] and r["calls"][-1] == (2, 32)  # 2 passes


def _forced_worker(rank, world, port):
    import os

    import torch

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer

    os.environ["DISTLEARN_POLICY"] = "full"
    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    tr = DataParallelTrainer(torch.nn.Linear(4, 2), tree, lr=0.1)
    ex = _FakeExecutor()
    tr.executor, tr.graph = ex, True
    tr._time_step_graph = lambda loader, reps: (_ for _ in ()).throw(AssertionError("measured a forced policy"))
    return {"policy": tr.select_policy(None), "calls": ex.calls}


def test_forced_policy_is_not_measured():
    for r in mp.run(_forced_worker, 2):
        assert r["policy"]["chosen"] == "full" and r["calls"] == [(3, 0)]


def _cap_worker(rank, world, port):
    import os

    import torch

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer

    os.environ.pop("DISTLEARN_CHANNEL_CAP", None)
    os.environ["DISTLEARN_CHANNEL_CAPS"] = "16,32"
    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    comm = tree.comm
    rebuilt = []
    comm.channel_cap = 32

    def set_cap(c):  # stands in for the RCCL communicator's rebuild (collective)
        rebuilt.append(c)
        comm.channel_cap = c

    comm.set_channel_cap = set_cap
    tr = DataParallelTrainer(torch.nn.Linear(4, 2), tree, lr=0.1)
    ex = _FakeExecutor()
    tr.executor, tr.graph = ex, True
    # rank-local ms per (policy, cap): the slowest rank makes reserve@16 the winner
    table = {(3, 0, 16): 0.40, (3, 0, 32): 0.36 + 0.1 * rank, (2, 16, 16): 0.35 + 0.01 * rank, (2, 32, 32): 0.38}
    seen = []

    def fake_time(loader, reps):
        key = ex.calls[-1] + (comm.channel_cap,)
        seen.append(key)
        return table[key]

    tr._time_step_graph = fake_time
    pol = tr.select_policy(None)
    return {"policy": pol, "seen": seen, "rebuilt": rebuilt, "final": ex.calls[-1], "cap": comm.channel_cap}


@pytest.mark.parametrize("world", [2])
def test_channel_cap_is_measured_with_the_policy(world):
    """the RCCL channel cap is not forced -- select_policy
    crosses the overlap policies with the candidate caps, rebuilds the
    communicator once per cap (caps outermost), the reserve policy leaves the
    cap's CUs free, and every rank takes the pair whose slowest rank is fastest."""
    res = mp.run(_cap_worker, world)
    for r in res:
        pol = r["policy"]
        assert set(pol["ms_per_step"]) == {"full@16", "reserve@16", "full@32", "reserve@32"}
        assert pol["chosen"] == "reserve@16" and pol["channel_cap"] == 16 and r["cap"] == 16
        assert r["final"] == (2, 16)
        fwd = [(3, 0, 16), (2, 16, 16), (3, 0, 32), (2, 32, 32)]
        assert r["seen"] == fwd + fwd[::-1]  # two passes, the second reversed
        assert r["rebuilt"] == [16, 32, 16]  # one rebuild per cap, then back to the winner's
        assert pol["candidates"]["reserve@32"] == {"dgrad_stages": 2, "cu_reserve": 32, "channel_cap": 32}


def _cap_mismatch_worker(rank, world, port):
    import os

    import torch

    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer

    os.environ.pop("DISTLEARN_CHANNEL_CAP", None)
    os.environ["DISTLEARN_CHANNEL_CAPS"] = "16,32" if rank == 0 else "16,64"
    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    tree.comm.set_channel_cap = lambda c: (_ for _ in ()).throw(AssertionError("rebuilt before agreeing"))
    tr = DataParallelTrainer(torch.nn.Linear(4, 2), tree, lr=0.1)
    tr.executor, tr.graph = _FakeExecutor(), True
    tr._time_step_graph = lambda loader, reps: 0.3
    try:
        tr.select_policy(None)
    except ValueError as e:
        return str(e)
    return "no error"


def test_channel_cap_lists_must_agree():
    """ranks whose environments give different cap lists fail with
    a clear error on every rank before any communicator rebuild."""
    for msg in mp.run(_cap_mismatch_worker, 2):
        assert "disagree on the channel caps" in msg
