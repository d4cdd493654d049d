"""AsyncEA: asynchronous Elastic-Averaging SGD with a parameter server.

Reference: lua/AsyncEA.lua:1-306 (+ examples/EASGD_{server,client,tester}.lua,
examples/AsyncEASGD.sh).  Roles and protocol:

* **server** holds the center variable; serves ONE client at a time (first
  come first served = the mutex, reference ``recvAny`` at :168-174): send the
  center, receive the client's elastic delta, ``center += delta``.
* **client** trains locally; every ``tau`` steps it enters the critical
  section, pulls the center, moves ``delta = alpha(p-c); p -= delta``
  (same fused kernel as AllReduceEA) and pushes ``delta``.
* **tester** periodically receives a snapshot of the center and evaluates it.

MI355X mapping:

* rank layout in one process group: rank 0 = server, ranks 1..numNodes =
  clients (``node`` = rank, like the reference's 1-based client ids), rank
  numNodes+1 = tester (optional);
* **control plane** (gloo, host): typed int64 messages
  ``[type, sender, seq, ...]`` -- ENTER/BYE (any-source receive; RCCL cannot
  express ``recvAny``), GRANT, TEST/STOP, ACK.  Every message carries a sequence
  number that is checked (replaces the reference's string asserts, :89,169,186);
* **data plane**: the center / delta payloads are point-to-point
  ``ncclSend/ncclRecv`` of the persistent flat buffers (C14/C15) on the GPU,
  gloo send/recv on CPU;
* **non-blocking tester** (reference defect: the server blocked on "Ack" for
  the tester's whole evaluation, :251-252): ``testNet`` only sends a new
  snapshot when the previous one has been acknowledged, and otherwise returns
  immediately;
* **explicit shutdown** (reference had none, numEpochs=inf loops forever):
  clients send BYE (:meth:`finishClient`), the server's :meth:`syncServer`
  returns False once every client said BYE, and :meth:`shutdown` stops the
  tester.
"""
from __future__ import annotations

from typing import Any, Optional

import torch
import torch.distributed as dist

from ..ops.flat import FlatParams, add_, elastic_step_
from ..utils.color_print import printClient, printServer
from .allreduce_ea import _FlatState
from .comm import MSG_LEN, Communicator
from .tree import Tree

# message types
ENTER, GRANT, BYE, TEST, STOP, ACK = 1, 2, 3, 4, 5, 6
# control-plane tags (separate channels, like the reference's ports P, P+i, P+N+1)
TAG_ENTER, TAG_GRANT, TAG_TEST, TAG_ACK = 11, 12, 13, 14

SERVER_RANK = 0


class AsyncEA:
    """``AsyncEA(server, serverBroadcast, client, clientBroadcast, serverTest,
    clientTest, numNodes, node, tau, alpha)`` (lua/AsyncEA.lua:6).

    The six channel arguments of the reference are replaced by one
    communicator: pass a :class:`Tree` / :class:`Communicator` as the first
    argument (the other five may be None), or use ``comm=``.
    """

    def __init__(self, server=None, serverBroadcast=None, client=None, clientBroadcast=None,  # noqa: N803
                 serverTest=None, clientTest=None, numNodes: int = 1, node: int = 0, tau: int = 10,  # noqa: N803
                 alpha: float = 0.2, comm: Optional[Communicator] = None):
        if comm is None:
            for c in (server, serverBroadcast, client, clientBroadcast, serverTest, clientTest):
                if isinstance(c, Tree):
                    comm = c.comm
                    break
                if isinstance(c, Communicator):
                    comm = c
                    break
        if comm is None:
            raise ValueError("AsyncEA needs a Tree/Communicator")
        self.comm = comm
        self.numNodes = int(numNodes)
        self.node = int(node)
        self.tau = int(tau)
        self.alpha = float(alpha)
        self.tester_rank = self.numNodes + 1 if comm.world_size > self.numNodes + 1 else None
        self.step = 0
        self.state: Optional[_FlatState] = None
        self.center = None
        self.delta = None
        self._seq = 0
        self._byes = 0
        self._test_inflight = False
        self._ack_work = None
        self._ack_buf = torch.zeros(MSG_LEN, dtype=torch.int64)
        self.syncs = 0

    # ------------------------------------------------------------- helpers
    def _one_time_init(self, params: Any):  # (:18-29)
        if self.state is None:
            self.state = _FlatState(params)
            self.center = self.state.flat.data.clone()
            self.delta = self.state.flat.data.clone()
        else:
            self.state.sync_in(params)

    @property
    def flat(self) -> FlatParams:
        return self.state.flat

    def _send_payload(self, buf: torch.Tensor, peer: int):
        self.comm.send(buf, peer)

    def _recv_payload(self, buf: torch.Tensor, peer: int):
        self.comm.recv(buf, peer)

    def _msg(self, typ: int, dst: int, tag: int, *extra):
        self._seq += 1
        self.comm.send_msg([typ, self.comm.rank, self._seq, *extra], dst, tag)

    def _expect(self, src, tag, *types):
        sender, m = self.comm.recv_msg(src, tag)
        if m[0] not in types:
            raise RuntimeError(f"AsyncEA protocol error: expected {types} on tag {tag}, got {m} from {sender}")
        if m[1] != sender:
            raise RuntimeError(f"AsyncEA protocol error: sender mismatch {m[1]} != {sender}")
        return sender, m

    def _is_sync_needed(self) -> bool:  # (:49-59)
        self.step += 1
        return self.step % self.tau == 0

    # --------------------------------------------------------------- client
    def initClient(self, params: Any) -> None:  # noqa: N802  (:64-78)
        self._one_time_init(params)
        self._recv_payload(self.center, SERVER_RANK)
        self.flat.data.copy_(self.center)
        self.flat.refresh_shadow()

    def syncClient(self, params: Any) -> bool:  # noqa: N802  (:134-146)
        self._one_time_init(params)
        if not self._is_sync_needed():
            return False
        printClient(self.node, "Waiting to sync")
        self._msg(ENTER, SERVER_RANK, TAG_ENTER)                 # clientEnterSync (:82-92)
        self._expect(SERVER_RANK, TAG_GRANT, GRANT)
        printClient(self.node, "Entered Sync")
        self._recv_payload(self.center, SERVER_RANK)             # clientGetCenter (:95-106)
        printClient(self.node, "Received center")
        f = self.flat                                            # calculateUpdateDiff (:109-119)
        elastic_step_(f.data, self.center, self.delta, self.alpha, shadow=f.shadow)
        self._send_payload(self.delta, SERVER_RANK)              # clientSendDiff (:122-132)
        self.syncs += 1
        return True

    def finishClient(self) -> None:  # noqa: N802
        """Tell the server this client is done (no reference equivalent)."""
        self._msg(BYE, SERVER_RANK, TAG_ENTER)

    # --------------------------------------------------------------- server
    def initServer(self, params: Any) -> None:  # noqa: N802  (:150-160)
        self._one_time_init(params)
        self.center.copy_(self.flat.data)
        for c in range(1, self.numNodes + 1):
            self._send_payload(self.center, c)

    def syncServer(self, params: Any) -> bool:  # noqa: N802  (:230-237)
        """Serve one client.  Returns False once every client said BYE."""
        self._one_time_init(params)
        while True:
            printServer("Server waiting to sync")
            sender, m = self._expect(None, TAG_ENTER, ENTER, BYE)  # serverEnterSync: recvAny (:163-177)
            if m[0] == BYE:
                self._byes += 1
                if self._byes >= self.numNodes:
                    return False
                continue
            break
        printServer(f"Current client is #{sender}")
        self._msg(GRANT, sender, TAG_GRANT)
        self._send_payload(self.center, sender)                   # serverSendCenter (:180-196)
        self._recv_payload(self.delta, sender)                    # serverGetUpdateDiff (:198-228)
        add_(self.center, self.delta)
        self.flat.data.copy_(self.center)
        self.flat.refresh_shadow()
        printServer(f"Received delta from client #{sender}")
        self.syncs += 1
        return True

    def _poll_ack(self, block: bool) -> None:
        if not self._test_inflight:
            return
        if self._ack_work is None:
            self._ack_work = dist.irecv(self._ack_buf, src=self.tester_rank, group=self.comm.ctrl, tag=TAG_ACK)
        if block:
            self._ack_work.wait()
        elif not self._ack_work.is_completed():
            return
        if int(self._ack_buf[0]) != ACK:
            raise RuntimeError(f"AsyncEA protocol error: expected ACK, got {self._ack_buf.tolist()}")
        self._ack_work = None
        self._test_inflight = False

    def testNet(self) -> bool:  # noqa: N802  (:239-258)
        """Send the tester a center snapshot unless it is still evaluating the
        previous one.  Returns True when a snapshot was sent."""
        if self.tester_rank is None:
            return False
        self._poll_ack(block=False)
        if self._test_inflight:
            return False
        self._msg(TEST, self.tester_rank, TAG_TEST)
        self._send_payload(self.center, self.tester_rank)
        self._test_inflight = True
        return True

    def shutdown(self) -> None:
        """Server: wait for the last ACK and stop the tester."""
        if self.tester_rank is not None:
            self._poll_ack(block=True)
            self._msg(STOP, self.tester_rank, TAG_TEST)

    # --------------------------------------------------------------- tester
    def initTester(self, params: Any) -> None:  # noqa: N802  (:261-265)
        self._one_time_init(params)

    def startTest(self, params: Any) -> bool:  # noqa: N802  (:268-285)
        """Receive the next snapshot into params; False when the server stops."""
        self._one_time_init(params)
        _, m = self._expect(SERVER_RANK, TAG_TEST, TEST, STOP)
        if m[0] == STOP:
            return False
        self._recv_payload(self.center, SERVER_RANK)
        self.flat.data.copy_(self.center)
        self.flat.refresh_shadow()
        return True

    def finishTest(self) -> None:  # noqa: N802  (:287-292)
        self._msg(ACK, SERVER_RANK, TAG_ACK)

    # python spellings
    init_server, init_client, init_tester = initServer, initClient, initTester
    sync_client, sync_server, test_net = syncClient, syncServer, testNet
    start_test, finish_test = startTest, finishTest
