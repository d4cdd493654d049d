"""N-rank RCCL data plane, one rank per GPU (the reference ran every
collective across real nodes: lua/AllReduceSGD.lua:20, lua/AllReduceEA.lua:41,
58-68, lua/AsyncEA.lua:87-130,155-159,183-228).

Every test is parameterised over the world size and skips cleanly when the box
has fewer GPUs (``torch.cuda.device_count() < N``); on a 1-GPU box only the
``gloo``-on-one-GPU rehearsal rows run (same worker code, data plane = gloo on
device tensors, hipGraph off: gloo is not capturable).  Oracles mirror the
reference's tests: bitwise-identical parameters after the uneven-step drain
(test/test_AllReduceSGD.lua:23-39), bit-identical EA centers
(test/test_AllReduceEA.lua:23-41), and the AsyncEA center == initial center +
every pushed delta.
"""
import os

import pytest
import torch

from tests import mp

pytestmark = pytest.mark.gpu

CASES = [("gloo", 2), ("rccl", 2), ("rccl", 4), ("rccl", 8)]


def _need(backend, world):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if backend == "rccl" and torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs (one rank per GPU), box has {torch.cuda.device_count()}")


def _setup(rank, world, port, backend):
    os.environ.setdefault("DISTLEARN_COMM_TIMEOUT", "120")
    import torch

    from torch_distlearn_amd import Tree

    dev = torch.device("cuda", rank if backend == "rccl" else 0)
    torch.cuda.set_device(dev)
    tree = Tree(rank + 1, world, host="127.0.0.1", port=port, device=dev, backend=backend)
    return dev, tree


# ---------------------------------------------------------------------------
def _collectives_worker(rank, world, port, backend):
    dev, tree = _setup(rank, world, port, backend)
    c = tree.comm
    out = {}
    x = torch.full((1 << 20,), float(rank + 1), device=dev)
    c.all_reduce(x)
    out["sum"] = float(x[0]), float(x[-1])
    b = torch.full((4099,), float(rank), device=dev, dtype=torch.bfloat16)
    c.broadcast(b, root=world - 1)
    out["bcast"] = float(b.float().min()), float(b.float().max())
    g = torch.empty(world * 5, device=dev)
    c.all_gather(g, torch.full((5,), float(rank), device=dev))
    out["gather"] = g.view(world, 5)[:, 0].tolist()
    if hasattr(c, "reduce_scatter"):
        rs = torch.empty(3, device=dev)
        c.reduce_scatter(rs, torch.arange(3 * world, device=dev, dtype=torch.float32))
        out["rs"] = rs.tolist()
    # ring p2p in one group (no deadlock: sends and receives are fused)
    s = torch.full((777,), float(rank), device=dev)
    r = torch.empty(777, device=dev)
    with c.group():
        c.send(s, (rank + 1) % world)
        c.recv(r, (rank - 1) % world)
    torch.cuda.synchronize()
    out["ring"] = float(r[0])
    c.check()
    return out


@pytest.mark.parametrize("backend,world", CASES)
def test_collectives(backend, world):
    _need(backend, world)
    res = mp.run(_collectives_worker, world, backend, timeout=300)
    tot = world * (world + 1) / 2
    for rank, o in enumerate(res):
        assert o["sum"] == (tot, tot)
        assert o["bcast"] == (world - 1, world - 1)
        assert o["gather"] == [float(r) for r in range(world)]
        if "rs" in o:
            assert o["rs"] == [float(world * (3 * rank + j)) for j in range(3)]
        assert o["ring"] == float((rank - 1) % world)


# ---------------------------------------------------------------------------
def _sgd_worker(rank, world, port, backend):
    dev, tree = _setup(rank, world, port, backend)
    from torch_distlearn_amd.data import DeviceLoader, PartitionedDataset
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet

    graph = backend == "rccl"
    model = CifarConvNet(seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.05, backend="hip", compute_dtype=torch.bfloat16,
                             bucket_bytes=1 << 20, graph=graph, max_batch=16)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(7 + rank)
    n_local = 16 * (6 + 3 * rank)  # uneven partitions -> uneven epochs -> drain
    imgs = torch.randint(0, 256, (n_local, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labs = torch.randint(0, 10, (n_local,), device=dev, generator=g)
    loader = DeviceLoader(PartitionedDataset(imgs, labs, device=dev), "permutation", 16, seed=rank)
    steps = []
    for _epoch in range(2):
        nsteps = loader.steps_per_epoch
        if graph:
            tr.run(loader, nsteps)   # unrolled hipGraphs with captured RCCL bucket all-reduces
        else:
            for _ in range(nsteps):
                tr.step(loader)
        steps.append(int(tr.sgd.stepsPerNode.sum()))
        tr.synchronize()  # drain (zero buckets) + winner broadcast
    torch.cuda.synchronize()
    tree.comm.check()
    return {"p": tr.flat.data.cpu(), "steps": steps, "nb": len(tr.bucketer.ranges),
            "finite": bool(torch.isfinite(tr.flat.data).all()), "captures": tr.captures}


@pytest.mark.parametrize("backend,world", CASES)
def test_sgd_hip_executor_buckets_graph_uneven(backend, world):
    _need(backend, world)
    res = mp.run(_sgd_worker, world, backend, timeout=600)
    assert all(r["finite"] for r in res)
    assert res[0]["nb"] == 3
    for rank, r in enumerate(res):
        assert r["steps"] == [6 + 3 * rank] * 2
        assert r["p"].tobytes() == res[0]["p"].tobytes(), f"rank {rank} params differ"


# ---------------------------------------------------------------------------
def _ea_worker(rank, world, port, backend):
    dev, tree = _setup(rank, world, port, backend)
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet

    model = CifarConvNet(seed=0).to(dev)
    tr = DataParallelTrainer(model, tree, lr=0.05, algo="ea", tau=3, alpha=0.3, backend="hip",
                             compute_dtype=torch.bfloat16, graph=backend == "rccl", max_batch=16)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(11 + rank)
    for _ in range(7 + 2 * rank):
        x = torch.randn(16, 32, 32, 3, device=dev, generator=g).to(torch.bfloat16)
        y = torch.randint(0, 10, (16,), device=dev, generator=g)
        tr.step(x, y)
    tr.synchronize()  # synchronizeCenter: drain + center scatter
    torch.cuda.synchronize()
    return {"c": tr.ea.center.cpu(), "p": tr.flat.data.cpu()}


@pytest.mark.parametrize("backend,world", CASES)
def test_ea_centers_bit_identical(backend, world):
    _need(backend, world)
    res = mp.run(_ea_worker, world, backend, timeout=600)
    for r in res:
        assert r["c"].tobytes() == res[0]["c"].tobytes()
        assert torch.isfinite(torch.from_numpy(r["p"])).all()


# ---------------------------------------------------------------------------
def _async_worker(rank, world, port, backend):
    dev, tree = _setup(rank, world, port, backend)
    from torch_distlearn_amd import AsyncEA, FlatParams
    from torch_distlearn_amd.utils.color_print import set_verbose

    set_verbose(False)
    torch.manual_seed(100 + rank)
    m = torch.nn.Sequential(torch.nn.Linear(300, 200), torch.nn.Linear(200, 10)).to(dev)
    flat = FlatParams(m, grads=False)
    nclients = world - 1
    ea = AsyncEA(tree, None, None, None, None, None, nclients, rank, 2, 0.25)
    if rank == 0:
        ea.initServer(flat)
        init = ea.center.clone()
        while ea.syncServer(flat):
            pass
        ea.shutdown()
        torch.cuda.synchronize()
        return {"init": init.cpu(), "center": ea.center.cpu(), "syncs": ea.syncs}
    ea.initClient(flat)
    sent = torch.zeros_like(ea.delta)
    g = torch.Generator(device=dev).manual_seed(rank)
    for _ in range(6 + rank):
        flat.data.add_(torch.randn(flat.data.shape, device=dev, generator=g) * 0.01)
        if ea.syncClient(flat):
            torch.cuda.current_stream().wait_stream(ea._ps)  # (test only) read delta after the push
            sent += ea.delta
    ea.finishClient()
    torch.cuda.synchronize()
    return {"sent": sent.cpu(), "syncs": ea.syncs}


@pytest.mark.parametrize("backend,world", CASES)
def test_async_ea_payload_stream(backend, world):
    _need(backend, world)
    res = mp.run(_async_worker, world, backend, timeout=600)
    server, clients = res[0], res[1:]
    assert server["syncs"] == sum(c["syncs"] for c in clients) > 0
    want = server["init"] + sum(c["sent"] for c in clients)
    got = server["center"]
    assert abs(got[64:] - want[64:]).max() < 1e-4


# ---------------------------------------------------------------------------
def test_watchdog_aborts_stuck_work(monkeypatch):
    """World-1 RCCL communicator with a 0.5 s timeout; a 2 s spin kernel
    (csrc/testing/diag.hip occupy_cus, light variant: every wave exits by
    itself) is handed to the watchdog: it must abort the communicator and
    every later call must raise CommError instead of hanging."""
    _need("gloo", 1)
    import time

    from torch_distlearn_amd import _native
    from torch_distlearn_amd.parallel.comm import CommError, RcclCommunicator

    monkeypatch.setenv("DISTLEARN_RCCL_WORLD1", "1")
    dev = torch.device("cuda", 0)
    T = _native.testing()
    comm = RcclCommunicator(0, 1, dev, ctrl_group=None, timeout_s=30.0)
    x = torch.ones(1024, device=dev)
    comm.all_reduce(x)
    torch.cuda.synchronize()
    time.sleep(0.3)
    assert comm.health() == "" and comm._c.pending() == 0  # healthy work retires
    comm.set_timeout(0.5)
    s = torch.cuda.Stream(device=dev)
    T.occupy_cus(-1, 2_000_000, 0, s.cuda_stream)
    comm.track(s)
    t0 = time.time()
    while comm.health() == "" and time.time() - t0 < 5:
        time.sleep(0.05)
    assert "did not complete within" in comm.health()
    assert time.time() - t0 < 1.5  # reported long before the 2 s kernel ends
    with pytest.raises(CommError):
        comm.all_reduce(x)
    with pytest.raises(CommError):
        comm.check()
    s.synchronize()  # the spin ends by itself
    comm.close()


def test_watchdog_times_grouped_collectives_from_group_end(monkeypatch):
    """RCCL launches grouped work only at the outermost ncclGroupEnd, so the
    watchdog's completion event for a collective issued inside ``group()`` must
    be recorded there: nothing is pending inside the group, one
    event per grouped op afterwards, and a grouped all-reduce queued behind a
    stuck kernel trips the timeout."""
    _need("gloo", 1)
    import time

    from torch_distlearn_amd import _native
    from torch_distlearn_amd.parallel.comm import RcclCommunicator

    monkeypatch.setenv("DISTLEARN_RCCL_WORLD1", "1")
    dev = torch.device("cuda", 0)
    T = _native.testing()
    comm = RcclCommunicator(0, 1, dev, ctrl_group=None, timeout_s=30.0)
    x = torch.ones(1024, device=dev)
    y = torch.ones(256, device=dev)
    s = torch.cuda.Stream(device=dev)
    T.occupy_cus(-1, 1_500_000, 0, s.cuda_stream)  # keeps s busy for 1.5 s
    with comm.group():
        comm.all_reduce(x, stream=s)
        comm.all_reduce(y, stream=s)
        assert comm._c.pending() == 0  # not launched yet: nothing to time
    assert comm._c.pending() == 2
    comm.set_timeout(0.5)
    t0 = time.time()
    while comm.health() == "" and time.time() - t0 < 5:
        time.sleep(0.05)
    assert "did not complete within" in comm.health()
    s.synchronize()
    comm.close()


# ---------------------------------------------------------------------------
# Every RCCL entry point at world 1.  NCCL/RCCL let a rank
# send to itself inside a group, so the p2p binding, all-gather,
# reduce-scatter and broadcast all run on the 1-GPU box through the same
# native communicator the N-GPU runs use (DISTLEARN_RCCL_WORLD1=1 forces the
# identity collectives through RCCL too).
def _world1(monkeypatch):
    _need("gloo", 1)
    from torch_distlearn_amd.parallel.comm import RcclCommunicator

    monkeypatch.setenv("DISTLEARN_RCCL_WORLD1", "1")
    dev = torch.device("cuda", 0)
    return dev, RcclCommunicator(0, 1, dev, ctrl_group=None, timeout_s=60.0)


def _drained(comm):
    import time

    t0 = time.time()
    while comm._c.pending() and time.time() - t0 < 5:
        time.sleep(0.02)
    return comm._c.pending() == 0 and comm._c.inflight() == 0


def test_rccl_world1_every_entry_point(monkeypatch):
    dev, comm = _world1(monkeypatch)
    g = torch.Generator(device=dev).manual_seed(3)
    # all-reduce (sum / max) and broadcast: identity at one rank, byte for byte
    x = torch.randn(1 << 16, device=dev, generator=g)
    x0 = x.clone()
    comm.all_reduce(x)
    comm.all_reduce(x, op="max")
    b = torch.randn(4099, device=dev, generator=g).to(torch.bfloat16)
    b0 = b.clone()
    comm.broadcast(b, root=0)
    # all-gather / reduce-scatter (world * n == n)
    src = torch.randint(-1000, 1000, (777,), device=dev, generator=g, dtype=torch.int64)
    gat = torch.empty_like(src)
    comm.all_gather(gat, src)
    rs_in = torch.randn(513, device=dev, generator=g)
    rs = torch.empty_like(rs_in)
    comm.reduce_scatter(rs, rs_in)
    # self send/recv inside a group (fp32, bf16, int64, uint8 payloads)
    pay = [torch.randn(12345, device=dev, generator=g), torch.randn(333, device=dev, generator=g).to(torch.bfloat16),
           torch.randint(0, 1 << 40, (99,), device=dev, generator=g, dtype=torch.int64),
           torch.randint(0, 255, (4096,), device=dev, generator=g, dtype=torch.uint8)]
    got = [torch.empty_like(p) for p in pay]
    with comm.group():
        for p, r in zip(pay, got):
            comm.send(p, 0)
            comm.recv(r, 0)
    torch.cuda.synchronize()
    assert torch.equal(x, x0) and torch.equal(b, b0)
    assert torch.equal(gat, src) and torch.equal(rs, rs_in)
    for p, r in zip(pay, got):
        assert torch.equal(p, r)
    assert _drained(comm) and comm.health() == ""
    comm.close()


def test_rccl_world1_p2p_inside_hipgraph(monkeypatch):
    """Grouped self send/recv captured into a hipGraph and replayed: each replay
    moves the CURRENT contents of the send buffer."""
    dev, comm = _world1(monkeypatch)
    s = torch.zeros(4096, device=dev)
    r = torch.full((4096,), -1.0, device=dev)
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up outside capture (connection setup)
        with comm.group():
            comm.send(s, 0)
            comm.recv(r, 0)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    from torch_distlearn_amd.engine import _capturing

    graph = torch.cuda.CUDAGraph()
    with _capturing(comm), torch.cuda.graph(graph, capture_error_mode="thread_local"):  # (the trainer's guard)
        with comm.group():
            comm.send(s, 0)
            comm.recv(r, 0)
    for k in range(3):
        s.fill_(float(k + 1))
        graph.replay()
        comm.track()
        torch.cuda.synchronize()
        assert float(r.min()) == float(r.max()) == float(k + 1)
    assert _drained(comm)
    # a graph holding captured RCCL work keeps a reference on the communicator:
    # ncclCommDestroy waits for it, so the graph goes first
    del graph
    torch.cuda.synchronize()
    comm.close()


def test_rccl_world1_async_payload_side_stream(monkeypatch):
    """The AsyncEA payload pattern (lua/AsyncEA.lua:95-132,180-228) at one
    rank: the center pull and the delta push are grouped self send/recv on a
    side stream, ordered against the compute stream by events only (no host
    synchronisation between the steps): compute writes the center, the side
    stream ships it into the client's buffer, compute derives the elastic
    delta from it, the side stream pushes the delta back, and the server's
    center += delta runs after the push."""
    dev, comm = _world1(monkeypatch)
    n = 300 * 200 + 200 * 10 + 210
    g = torch.Generator(device=dev).manual_seed(9)
    main = torch.cuda.current_stream()
    ps = torch.cuda.Stream(device=dev)
    center = torch.randn(n, device=dev, generator=g)   # server's center
    params = torch.randn(n, device=dev, generator=g)   # client's replica
    c_recv = torch.empty(n, device=dev)                # client's copy of the center
    delta = torch.empty(n, device=dev)
    d_recv = torch.empty(n, device=dev)                # server's receive buffer
    alpha = 0.25
    want_center, want_params = center.clone(), params.clone()
    for _ in range(5):
        want_delta = alpha * (want_params - want_center)
        want_params -= want_delta
        want_center += want_delta
        center_ready = torch.cuda.Event()
        center_ready.record(main)
        ps.wait_event(center_ready)
        with torch.cuda.stream(ps):  # pull: server -> client
            with comm.group():
                comm.send(center, 0, stream=ps)
                comm.recv(c_recv, 0, stream=ps)
        pulled = torch.cuda.Event()
        pulled.record(ps)
        main.wait_event(pulled)
        torch.sub(params, c_recv, out=delta).mul_(alpha)   # calculateUpdateDiff
        params.sub_(delta)
        delta_ready = torch.cuda.Event()
        delta_ready.record(main)
        ps.wait_event(delta_ready)
        with torch.cuda.stream(ps):  # push: client -> server
            with comm.group():
                comm.send(delta, 0, stream=ps)
                comm.recv(d_recv, 0, stream=ps)
        pushed = torch.cuda.Event()
        pushed.record(ps)
        main.wait_event(pushed)
        center.add_(d_recv)                                 # serverGetUpdateDiff
    torch.cuda.synchronize()
    torch.testing.assert_close(center, want_center, rtol=0, atol=1e-5)
    torch.testing.assert_close(params, want_params, rtol=0, atol=1e-5)
    assert _drained(comm)
    comm.close()


def test_rccl_abort_waits_for_open_group(monkeypatch):
    """an abort while a host call holds the communicator (here: an
    open group) must not free it under that call; the abort completes at the
    group's end and later calls raise CommError."""
    from torch_distlearn_amd.parallel.comm import CommError

    dev, comm = _world1(monkeypatch)
    x = torch.ones(64, device=dev)
    r = torch.empty(64, device=dev)
    with comm.group():
        comm.send(x, 0)
        comm.recv(r, 0)
        assert comm._c.inflight() == 1  # the group holds the handle until its end
        comm._c.abort()                 # watchdog/user abort from "another thread"
        assert comm._c.inflight() == 1 and "aborted" in comm.health()
        with pytest.raises(CommError):
            comm.send(x, 0)             # no new call on a failed communicator
    # group end issued the matched pair on the still-valid handle, then aborted it
    assert comm._c.inflight() == 0
    torch.cuda.synchronize()
    with pytest.raises(CommError):
        comm.all_reduce(x)
    comm.close()


def test_rccl_watchdog_pause_is_synchronous(monkeypatch):
    """pause_watch(True) -- what every hipGraph capture
    runs first (engine._capturing) -- returns only when no watchdog poll is in
    progress, and no poll runs until resumed (csrc/comm/pause_gate.h; the
    handshake itself is TSan-tested on the CPU, tests/unit/test_capture_guard.py)."""
    import time

    dev, comm = _world1(monkeypatch)
    x = torch.ones(1024, device=dev)
    comm.all_reduce(x)
    time.sleep(0.3)  # the watchdog polls every 50 ms
    assert comm._c.polls() > 0
    for _ in range(5):
        comm.pause_watch(True)
        n = comm._c.polls()
        time.sleep(0.2)
        assert comm._c.polls() == n
        comm.pause_watch(False)
        time.sleep(0.2)
        assert comm._c.polls() > n
    assert _drained(comm) and comm.health() == ""
    comm.close()


# ---------------------------------------------------------------------------
def _async_hip_worker(rank, world, port, backend, unrolled):
    os.environ["DISTLEARN_REDUCE_ATOMIC"] = "0"  # deterministic kernels: the two runs compare bitwise
    dev, tree = _setup(rank, world, port, backend)
    from torch_distlearn_amd import AsyncEA, FlatParams
    from torch_distlearn_amd.data import DeviceLoader, PartitionedDataset
    from torch_distlearn_amd.engine import DataParallelTrainer
    from torch_distlearn_amd.models import CifarConvNet
    from torch_distlearn_amd.utils.color_print import set_verbose

    set_verbose(False)
    model = CifarConvNet(seed=0).to(dev)
    ea = AsyncEA(tree, None, None, None, None, None, world - 1, rank, 3, 0.3)
    if rank == 0:
        flat = FlatParams(model, grads=False)
        ea.initServer(flat)
        while ea.syncServer(flat):
            pass
        torch.cuda.synchronize()
        return {"center": ea.center.cpu(), "syncs": ea.syncs}
    tr = DataParallelTrainer(model, tree, lr=0.02, algo="async", tau=3, alpha=0.3, backend="hip",
                             compute_dtype=torch.bfloat16, graph=True, max_batch=16, async_ea=ea)
    tr.synchronize_parameters()
    g = torch.Generator(device=dev).manual_seed(5)
    imgs = torch.randint(0, 256, (16 * 8, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labs = torch.randint(0, 10, (16 * 8,), device=dev, generator=g)
    loader = DeviceLoader(PartitionedDataset(imgs, labs, device=dev), "permutation", 16, seed=1)
    if unrolled:
        tr.run(loader, 11, unroll=4)
    else:
        for _ in range(11):
            tr.step(loader)
    tr.finish()
    torch.cuda.synchronize()
    return {"p": tr.flat.data.cpu(), "syncs": ea.syncs, "step": ea.step, "keys": sorted(str(k) for k in tr._multi),
            "slabs": tr._slabs is not None, "side": tr._side is not None}


def test_async_ea_hip_client_unrolled(monkeypatch):
    """an AsyncEA client on the MI355X hot path --
    DataParallelTrainer(algo="async", backend="hip", graph=True) with the
    tau-1 local steps between two syncs replayed as ONE hipGraph (engine.run)
    trains BITWISE like one captured step at a time (deterministic kernels),
    against a real server rank (1 server + 1 client sharing the GPU, gloo
    payloads: RCCL refuses two ranks on one GPU)."""
    _need("gloo", 2)
    outs = [mp.run(_async_hip_worker, 2, "gloo", u, timeout=600) for u in (False, True)]
    (s0, c0), (s1, c1) = outs
    assert c0["syncs"] == c1["syncs"] == 3 == s0["syncs"] == s1["syncs"] and c0["step"] == c1["step"] == 11
    assert "('async', 2)" in c1["keys"] and c1["slabs"] and not c1["side"]
    assert c0["p"].tobytes() == c1["p"].tobytes()
    assert s0["center"].tobytes() == s1["center"].tobytes()
