"""AsyncEA parameter server (no reference test exists).

1 server + 2 clients + 1 tester on gloo.  Checks: clients start from the
server's center, the server's final center == initial center + every delta
the clients pushed, server sync count == sum of client syncs, the tester
receives snapshots without blocking the server, and shutdown terminates every
role.
"""
import pytest
import torch

from tests import mp

NUM_CLIENTS = 2
TAU = 3


def _async_worker(rank, world, port, wire="fp32"):
    from torch_distlearn_amd import AsyncEA, Tree

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    torch.manual_seed(100 + rank)  # deliberately different init per role
    params = {"w": torch.randn(6), "b": torch.randn(3)}
    ea = AsyncEA(tree, None, None, None, None, None, NUM_CLIENTS, rank, TAU, 0.3, delta_wire=wire)
    if rank == 0:  # server
        ea.initServer(params)
        init = ea.center.clone()
        tests = 0
        while ea.syncServer(params):
            if ea.syncs % 2 == 0:
                tests += ea.testNet()
        ea.shutdown()
        return {"role": "server", "init": init, "center": ea.center.clone(), "syncs": ea.syncs, "tests": tests}
    if rank <= NUM_CLIENTS:  # client
        ea.initClient(params)
        start = torch.cat([params["b"], params["w"]]).clone()
        sent = torch.zeros_like(ea.delta)
        conserved = []
        for step in range(20 + 4 * rank):
            g = {"w": torch.randn(6) * 0.1, "b": torch.randn(3) * 0.1}
            before = ea.flat.data.clone() if ea.state is not None else None
            if ea.syncClient(params):
                sent += ea.delta
                if wire == "bf16":  # what went on the wire is bf16, and the client moved by exactly it
                    assert torch.equal(ea.delta[64:], ea.delta16[64:].float())
                    conserved.append(float((before[64:] - ea.flat.data[64:] - ea.delta[64:]).abs().max()))
            params["w"].add_(-0.1 * g["w"])
            params["b"].add_(-0.1 * g["b"])
            params["w"].add_(-0.1 * g["w"])
            params["b"].add_(-0.1 * g["b"])
        ea.finishClient()
        return {"role": "client", "start": start, "sent": sent, "syncs": ea.syncs, "conserved": conserved}
    # tester
    ea.initTester(params)
    n = 0
    while ea.startTest(params):
        n += 1
        ea.finishTest()
    return {"role": "tester", "snapshots": n}


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_async_ea_protocol(wire):
    """fp32 and bf16 delta wires: with bf16 the server's center is still the
    initial center + every delta the clients moved by (the rounded ones)."""
    world = NUM_CLIENTS + 2
    res = mp.run(_async_worker, world, wire, timeout=180)
    server, clients, tester = res[0], res[1:1 + NUM_CLIENTS], res[-1]
    assert server["syncs"] == sum(c["syncs"] for c in clients)
    assert all(c["syncs"] == (20 + 4 * (i + 1)) // TAU for i, c in enumerate(clients))
    # every client started from the server's initial center (header region skipped)
    init = server["init"]
    for c in clients:
        s = c["start"]  # sorted keys: "b" at flat offset 64, "w" at 128
        assert (s[0:3] == init[64:67]).all() and (s[3:9] == init[128:134]).all()
    total_sent = sum(c["sent"] for c in clients)
    want = init + total_sent
    got = server["center"]
    # compare the parameter regions (offsets 64..67 for "b", 128..134 for "w")
    for lo, hi in ((64, 67), (128, 134)):
        assert abs(got[lo:hi] - want[lo:hi]).max() < 1e-5
    assert tester["snapshots"] == server["tests"] and tester["snapshots"] >= 1
    if wire == "bf16":
        assert all(c["conserved"] and max(c["conserved"]) < 1e-6 for c in clients)
