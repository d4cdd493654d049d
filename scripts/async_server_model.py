"""AsyncEA with 1 server + k clients: what one server sync costs, measured at
world 1 on one MI355X, and the throughput model built from it (VERDICT r4
item 4; protocol: lua/AsyncEA.lua:163-228).

Measured here (rank 0 on the GPU, rank 1 a CPU process for the control plane):
  * ctrl   -- ENTER -> GRANT round trip over the gloo control plane (localhost
              TCP), the host part of clientEnterSync / serverEnterSync;
  * p2p    -- the center pull and the delta push of one sync as RCCL self
              send/recv pairs (grouped, world 1) on the payload stream: RCCL's
              issue cost plus an on-device copy of the 17.3 MB flat buffer;
  * apply  -- the server's center += delta, params <- center, bf16 shadow
              (add_, copy_, cast: the GPU work of serverGetUpdateDiff);
  * elastic -- the client's fused elastic kernel (calculateUpdateDiff).
Modelled (no second GPU here): the xGMI transfer of the 17.3 MB payload each
way over the single link between the server and that client.

The server handles one client at a time; its per-sync service time is
  T_s = ctrl + max(p2p, bytes / link_bw) + max(p2p_push, push_bytes / link_bw) + apply
(the center pull is fp32; the delta push is fp32 or, with AsyncEA
delta_wire="bf16", half the bytes -- the client then rounds its delta and
moves by the rounded one, the server casts it back: both measured here)
(the payload stream serialises the pull and the push; the host loop moves on
to the next ENTER while the GPU still applies the delta, so apply only counts
when the GPU is the bottleneck).  A client syncs every tau steps; alone it
would cycle in T_c = tau * t_step + T_s.  With k clients the server is busy
a fraction rho = k * T_s / T_c; once rho >= 1 the clients queue on the mutex
and the node's throughput saturates at tau * B / T_s images/s.

    python scripts/async_server_model.py [--tau 10] [--clients 7] [--step-ms 0.303]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

N_PARAMS = 4_328_970  # CIFAR convnet (examples/cifar10.lua:108-133)


def ctrl_peer(rank, port, reps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    from torch_distlearn_amd.parallel.comm import ProcessGroupCommunicator

    c = ProcessGroupCommunicator(dist.group.WORLD)
    if rank == 1:  # client: ENTER, wait for GRANT
        for i in range(reps + 10):
            if i == 10:
                t0 = time.perf_counter()
            c.send_msg([1, 1, i], 0, tag=11)
            c.recv_msg(0, tag=12)
        q.put((time.perf_counter() - t0) / reps * 1e6)
    else:  # server: recvAny ENTER, GRANT
        for i in range(reps + 10):
            c.recv_msg(None, tag=11)
            c.send_msg([2, 0, i], 1, tag=12)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tau", type=int, default=10)
    ap.add_argument("--clients", type=int, default=7)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--step-ms", type=float, default=0.303, help="client step time (bench.py --algo sgd, 1 GPU)")
    ap.add_argument("--link-GBps", type=float, nargs="+", default=[64.0, 153.0],
                    help="xGMI bandwidth of one server<->client link per direction (assumptions to model)")
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    # control plane: two CPU processes over gloo
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29000 + os.getpid() % 1000
    ps = [ctx.Process(target=ctrl_peer, args=(r, port, a.reps, q)) for r in range(2)]
    for p in ps:
        p.start()
    ctrl_us = q.get(timeout=300)
    for p in ps:
        p.join(timeout=60)

    os.environ["DISTLEARN_RCCL_WORLD1"] = "1"
    from torch_distlearn_amd.ops.flat import add_, cast_, elastic_step_, elastic_step_wire16_
    from torch_distlearn_amd.parallel.comm import RcclCommunicator

    dev = torch.device("cuda", 0)
    comm = RcclCommunicator(0, 1, dev, ctrl_group=None, timeout_s=120.0)
    n = (N_PARAMS + 63) // 64 * 64 + 64 * 18  # the flat buffer (aligned leaves + header)
    center = torch.randn(n, device=dev)
    params = torch.randn(n, device=dev)
    delta = torch.empty(n, device=dev)
    recv = torch.empty(n, device=dev)
    d16 = torch.empty(n, device=dev, dtype=torch.bfloat16)
    recv16 = torch.empty(n, device=dev, dtype=torch.bfloat16)
    shadow = torch.empty(n, device=dev, dtype=torch.bfloat16)
    pstream = torch.cuda.Stream(device=dev)

    def timed(fn, reps):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        for _ in range(reps):
            fn()
        e1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    def p2p():  # one payload transfer (pull or push) on the payload stream
        pstream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(pstream):
            with comm.group():
                comm.send(center, 0, stream=pstream)
                comm.recv(recv, 0, stream=pstream)
        torch.cuda.current_stream().wait_stream(pstream)

    def p2p16():  # the bf16 delta push
        pstream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(pstream):
            with comm.group():
                comm.send(d16, 0, stream=pstream)
                comm.recv(recv16, 0, stream=pstream)
        torch.cuda.current_stream().wait_stream(pstream)

    def apply():
        add_(center, recv)
        params.copy_(center)
        cast_(shadow, params)

    def apply16():  # serverGetUpdateDiff with the bf16 wire (async_ea.syncServer)
        cast_(recv, recv16)
        apply()

    def elastic():
        elastic_step_(params, center, delta, 0.2, shadow=shadow)

    def elastic16():  # async_ea.syncClient with the bf16 wire: one fused kernel
        elastic_step_wire16_(params, center, delta, d16, 0.2, shadow=shadow)

    p2p_us = timed(p2p, a.reps)
    p2p16_us = timed(p2p16, a.reps)
    apply_us = timed(apply, a.reps)
    apply16_us = timed(apply16, a.reps)
    elastic_us = timed(elastic, a.reps)
    elastic16_us = timed(elastic16, a.reps)
    comm.close()

    nbytes = n * 4
    t_step_us = a.step_ms * 1e3
    rows = []
    for wire in ("fp32", "bf16"):
        push_bytes, push_us = (nbytes, p2p_us) if wire == "fp32" else (nbytes // 2, p2p16_us)
        app_us, el_us = (apply_us, elastic_us) if wire == "fp32" else (apply16_us, elastic16_us)
        for bw in a.link_GBps:
            xfer = nbytes / (bw * 1e9) * 1e6
            xpush = push_bytes / (bw * 1e9) * 1e6
            t_s = ctrl_us + max(p2p_us, xfer) + max(push_us, xpush) + app_us
            t_c = a.tau * t_step_us + t_s + el_us
            rho = a.clients * t_s / t_c
            # clients alone: k * tau * B / T_c; server-bound: tau * B / T_s
            ips_free = a.clients * a.tau * a.batch / (t_c * 1e-6)
            ips_cap = a.tau * a.batch / (t_s * 1e-6)
            rows.append({"delta_wire": wire, "link_GBps": bw, "xfer_us_pull": round(xfer, 1),
                         "xfer_us_push": round(xpush, 1), "server_us_per_sync": round(t_s, 1),
                         "client_cycle_us": round(t_c, 1), "server_utilisation": round(rho, 3),
                         "node_img_per_s": round(min(ips_free, ips_cap), 0),
                         "bound": "server" if rho >= 1 else "clients", "clients_for_saturation": round(t_c / t_s, 2)})
    out = {"measured_world1": {"ctrl_roundtrip_us": round(ctrl_us, 1), "p2p_self_us": round(p2p_us, 1),
                               "p2p_self_bf16_us": round(p2p16_us, 1), "server_apply_us": round(apply_us, 1),
                               "server_apply_bf16_us": round(apply16_us, 1), "client_elastic_us": round(elastic_us, 1),
                               "client_elastic_bf16_us": round(elastic16_us, 1),
                               "payload_MB": round(nbytes / 1e6, 2)},
           "tau": a.tau, "clients": a.clients, "batch": a.batch, "client_step_ms": a.step_ms, "model": rows}
    txt = json.dumps(out, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
