"""DataParallelTrainer end-to-end on gloo (world 2/3): each rank trains on its
own data; with AllReduceSGD the parameters stay BITWISE identical on every
rank after every step (bucketed all-reduce issued from post-accumulate-grad
hooks, participation slot n, fused 1/n + SGD) and equal a single-process
reference trained on the concatenated batch's mean gradient."""
import pytest
import torch

from tests import mp


def _worker(rank, world, port, algo, uneven):
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import MnistConvNet

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    model = MnistConvNet(seed=0)
    tr = DataParallelTrainer(model, tree, lr=0.05, algo=algo, tau=2, alpha=0.3, compute_dtype=torch.float32,
                             bucket_bytes=8 << 10)
    tr.synchronize_parameters()
    g = torch.Generator().manual_seed(rank)
    steps = 5 + (rank if uneven else 0)
    for _ in range(steps):
        x = torch.randn(4, 1024, generator=g)
        y = torch.randint(0, 10, (4,), generator=g)
        tr.step(x, y)
    tr.synchronize()
    return {"p": tr.flat.data.clone(), "nb": len(tr.bucketer.ranges) if tr.bucketer else 0,
            "c": tr.ea.center.clone() if tr.ea is not None else None}


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("uneven", [False, True])
def test_engine_sgd_bitwise(world, uneven):
    res = mp.run(_worker, world, "sgd", uneven)
    assert res[0]["nb"] > 1, "several buckets expected (overlap path)"
    for r in res[1:]:
        assert (r["p"] == res[0]["p"]).all()


def test_engine_sgd_matches_single_process_mean_gradient():
    """2 ranks x batch 4 == 1 process on the 8-sample batch (mean loss)."""
    from torch_distlearn_amd.models import MnistConvNet

    res = mp.run(_worker, 2, "sgd", False)
    m = MnistConvNet(seed=0)
    opt = torch.optim.SGD(m.parameters(), lr=0.05)
    gens = [torch.Generator().manual_seed(r) for r in range(2)]
    for _ in range(5):
        xs, ys = [], []
        for g in gens:
            xs.append(torch.randn(4, 1024, generator=g))
            ys.append(torch.randint(0, 10, (4,), generator=g))
        opt.zero_grad()
        m.loss(m(torch.cat(xs)), torch.cat(ys)).backward()
        opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    from torch_distlearn_amd import FlatParams

    f = FlatParams(MnistConvNet(seed=0), grads=False)
    p0 = torch.from_numpy(res[0]["p"])
    got = torch.cat([p0[o:o + n] for o, n in zip(f.offsets, f.numels)])
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)


def test_engine_ea_centers_agree():
    res = mp.run(_worker, 2, "ea", True)
    # after synchronizeCenter the centers are broadcast from node 1: bit-identical
    # (lua/AllReduceEA.lua:74-83); params stay elastic (they differ) but finite
    assert res[0]["c"].tobytes() == res[1]["c"].tobytes()
    assert all(torch.isfinite(torch.from_numpy(r["p"])).all() for r in res)
    assert (res[0]["p"] != res[1]["p"]).any(), "uneven elastic runs should leave distinct local params"
    # the center header (participation count) never leaks into the body
    assert (res[0]["c"][:64] == res[0]["p"][:64]).all()


def _debug_worker(rank, world, port, perturb):
    import os

    os.environ["DISTLEARN_DEBUG_SYNC"] = "1"
    from torch_distlearn_amd import AllReduceSGD, Tree
    from torch_distlearn_amd.utils.debug import assert_replicas_in_sync

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    params = [torch.arange(5.0)]
    sgd = AllReduceSGD(tree)
    sgd.synchronizeParameters(params)  # runs the checksum check (in sync)
    if perturb and rank == 1:
        params[0][2] += 1e-3
    try:
        assert_replicas_in_sync(tree, params[0])
        return "ok"
    except RuntimeError as e:
        return "diverged" if "divergence" in str(e) else repr(e)


def test_replica_divergence_detection():
    assert mp.run(_debug_worker, 2, False) == ["ok", "ok"]
    assert mp.run(_debug_worker, 2, True) == ["diverged", "diverged"]


def _seq_worker(rank, world, port, algo, inject):
    """Uneven epochs through the trainer with DISTLEARN_DEBUG_SYNC=1: the
    collective-sequence hashes agree at every epoch synchronisation (after the
    drain).  ``inject``: in epoch 2 node 2 issues one all-reduce with another
    op than the others' (gloo runs it without hanging -- the silent kind of
    divergence); the next synchronisation must raise CommError."""
    import os

    os.environ["DISTLEARN_DEBUG_SYNC"] = "1"
    from torch_distlearn_amd import Tree
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import MnistConvNet
    from torch_distlearn_amd.parallel.comm import CommError

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    tr = DataParallelTrainer(MnistConvNet(seed=0), tree, lr=0.05, algo=algo, tau=2, alpha=0.3,
                             compute_dtype=torch.float32, bucket_bytes=8 << 10)
    tr.synchronize_parameters()
    g = torch.Generator().manual_seed(rank)
    seen = []
    for epoch in range(3):
        if inject and epoch == 1:  # (aligned: every rank is at the same collective after a sync)
            t = torch.ones(16)
            tree.comm.all_reduce(t, "max" if rank == 1 else "sum")
        for _ in range(3 + (rank + epoch) % world):  # uneven per node and per epoch
            tr.step(torch.randn(4, 1024, generator=g), torch.randint(0, 10, (4,), generator=g))
        try:
            tr.synchronize()
        except CommError as e:
            return {"raised": str(e), "epoch": epoch, "seen": seen}
        seen.append(tree.comm.seq_state()[1])
    return {"raised": None, "seen": seen}


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("algo", ["sgd", "ea"])
def test_collective_sequence_hash_agrees_on_uneven_epochs(world, algo):
    """every rank's hash of the collectives it issued
    (graph replays included) agrees at the epoch synchronisation, uneven
    epochs and drains notwithstanding."""
    res = mp.run(_seq_worker, world, algo, False)
    for r in res:
        assert r["raised"] is None and len(r["seen"]) == 3
        assert r["seen"] == res[0]["seen"] and r["seen"][0] > 0


@pytest.mark.parametrize("world", [2, 4])
def test_collective_sequence_divergence_raises(world):
    """An injected collective that differs on one rank raises CommError on
    every rank at the next synchronisation, naming the nodes."""
    res = mp.run(_seq_worker, world, "sgd", True)
    for r in res:
        assert r["raised"] is not None and r["epoch"] == 1, r
        assert "collective sequence diverged" in r["raised"] and "nodes [2]" in r["raised"]


def test_sequence_record_and_replay():
    """A captured graph's collectives are recorded, not counted; each replay
    counts them (the engine's _seq_record / _replay)."""
    import os

    from torch_distlearn_amd.parallel.comm import Communicator

    os.environ["DISTLEARN_DEBUG_SYNC"] = "1"
    try:
        a, b = Communicator(), Communicator()
        t = torch.zeros(8)
        with a.seq_record() as rec:
            a._note("all_reduce", t, 0)
            a._note("broadcast", t, 1)
        assert a.seq_state()[1] == 0 and len(rec) == 2
        a.seq_replay(rec, times=3)
        for _ in range(3):
            b._note("all_reduce", t, 0)
            b._note("broadcast", t, 1)
        assert a.seq_state() == b.seq_state()
        b._note("broadcast", t, 0)  # another root: another hash
        a._note("broadcast", t, 1)
        assert a.seq_state()[1] == b.seq_state()[1] and a.seq_state()[0] != b.seq_state()[0]
    finally:
        os.environ.pop("DISTLEARN_DEBUG_SYNC", None)
