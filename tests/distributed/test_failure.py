"""Failure detection (the reference has none: a dead peer hangs
every tree operation forever).  A stuck or dead peer must turn into a
:class:`CommError` on the survivors within the configured timeout
(``DISTLEARN_COMM_TIMEOUT`` / ``--commTimeout``), for the synchronous
algorithms' collectives and for the AsyncEA server/client/tester roles."""
import os
import time

import pytest
import torch

from tests import mp

TIMEOUT = 4.0


def _collective_worker(rank, world, port, mode):
    os.environ["DISTLEARN_COMM_TIMEOUT"] = str(TIMEOUT)
    from torch_distlearn_amd import AllReduceSGD, Tree
    from torch_distlearn_amd.parallel.comm import CommError

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    sgd = AllReduceSGD(tree)
    grads = [torch.ones(5)]
    sgd.sumAndNormalizeGradients(grads)  # one healthy round
    if rank == world - 1:
        if mode == "die":
            os._exit(3)
        time.sleep(3 * TIMEOUT)  # stuck peer
        return "stuck"
    t0 = time.time()
    try:
        for _ in range(3):
            sgd.sumAndNormalizeGradients(grads)
        return "no error"
    except CommError as e:
        return ("CommError", time.time() - t0, str(e))


@pytest.mark.parametrize("mode", ["stuck", "die"])
def test_stuck_or_dead_peer_is_bounded(mode):
    world = 3
    res = mp.run(_collective_worker, world, mode, timeout=60, dead=(world - 1,) if mode == "die" else ())
    for r in res[:-1]:
        assert r[0] == "CommError", r
        assert r[1] < TIMEOUT + 6, f"failure surfaced after {r[1]:.1f} s"


def _async_worker(rank, world, port, victim):
    os.environ["DISTLEARN_COMM_TIMEOUT"] = str(TIMEOUT)
    from torch_distlearn_amd import AsyncEA, Tree
    from torch_distlearn_amd.parallel.comm import CommError

    tree = Tree(rank + 1, world, host="127.0.0.1", port=port)
    params = [torch.randn(6)]
    nclients = world - 2
    ea = AsyncEA(tree, None, None, None, None, None, nclients, rank, 2, 0.3)
    t0 = None
    try:
        if rank == 0:
            ea.initServer(params)
            t0 = time.time()
            while ea.syncServer(params):
                ea.testNet()
            ea.shutdown()
            return "server finished"
        if rank <= nclients:
            ea.initClient(params)
            for step in range(30):
                if rank == victim and step == 5:
                    os._exit(3)  # client dies mid-run, without BYE
                ea.syncClient(params)
                time.sleep(0.01)
            ea.finishClient()
            return "client finished"
        ea.initTester(params)
        t0 = time.time()
        while ea.startTest(params):
            ea.finishTest()
        return "tester finished"
    except CommError as e:
        return ("CommError", None if t0 is None else time.time() - t0, str(e))


def test_async_ea_dead_client_stops_server_and_tester():
    """A client dies after a few syncs: the server stops waiting for it and
    raises (naming it), the tester stops too -- all within the timeout, no
    hang (the reference's server loops forever on recvAny)."""
    world, victim = 4, 2   # server, clients 1-2, tester
    res = mp.run(_async_worker, world, victim, timeout=90, dead=(victim,))
    server, tester = res[0], res[-1]
    assert res[1] == "client finished"
    assert server[0] == "CommError" and "[2]" in server[2], server
    assert tester[0] == "CommError" or tester == "tester finished", tester
