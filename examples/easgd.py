#!/usr/bin/env python3
"""Asynchronous EASGD with a parameter server (reference: examples/EASGD_server.lua,
EASGD_client.lua, EASGD_tester.lua, AsyncEASGD.sh).

Roles share one process group: rank 0 = server, ranks 1..numNodes = clients,
rank numNodes+1 = tester (optional).  ``--role auto`` derives the role from
$RANK (what the launcher sets); ``--server`` / ``--tester`` force it like the
reference's flags.

* client: grads = df(params, x, y); ``syncClient`` every ``--communicationTime``
  steps (elastic move against the server's center); then the SGD step with the
  pre-move grads (EASGD_client.lua:106-117).  Sends BYE when done.  On a GPU
  (CIFAR-10) the client trains through ``DataParallelTrainer(algo="async",
  backend="hip", graph=True)``: the hand-written kernels, a device-side
  sampler, and the tau-1 local steps between two syncs replayed as ONE
  hipGraph (engine.run); it prints its images/s.
* server: ``syncServer`` until every client said BYE; every ``--testTime``
  syncs ``testNet`` hands the tester a center snapshot WITHOUT blocking on the
  tester's evaluation (reference defect fixed).
* tester: evaluates each snapshot on the train/test partitions (the HIP
  executor's forward on a GPU, BatchNorm on the batch statistics like the
  reference's functional model, examples/Model.lua:56-66), appends
  "Training Error"/"Test Error" to ``Results/<save>/ErrorRate.log``, logs to
  ``Log.txt`` and writes the ``Net``/``optState`` checkpoint.

    python -m torch_distlearn_amd.launch --nproc 4 --no-node-flags examples/easgd.py --numNodes 2
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from torch_distlearn_amd import AsyncEA, FlatParams, Tree  # noqa: E402
from torch_distlearn_amd.checkpoint import load_checkpoint, results_dir, save_checkpoint  # noqa: E402
from torch_distlearn_amd.data import Dataset, DeviceLoader  # noqa: E402
from torch_distlearn_amd.engine import DataParallelTrainer, predict_module  # noqa: E402
from torch_distlearn_amd.launch import device_of  # noqa: E402
from torch_distlearn_amd.models import CifarConvNet, MnistConvNet, make_executor  # noqa: E402
from torch_distlearn_amd.parallel.comm import CommError  # noqa: E402
from torch_distlearn_amd.utils.color_print import set_verbose  # noqa: E402
from torch_distlearn_amd.utils.metrics import ConfusionMatrix, Logger  # noqa: E402


def parse():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--nodeIndex", type=int, default=1, help="client index (1-based)")
    ap.add_argument("--numNodes", type=int, default=1, help="number of clients")
    ap.add_argument("--role", default="auto", choices=["auto", "server", "client", "tester"])
    ap.add_argument("--server", action="store_true")
    ap.add_argument("--tester", action="store_true")
    ap.add_argument("--noTester", action="store_true", help="run without a tester process")
    ap.add_argument("--batchSize", type=int, default=128)
    ap.add_argument("--learningRate", type=float, default=0.01)
    ap.add_argument("--numEpochs", type=int, default=1)
    ap.add_argument("--maxSteps", type=int, default=0)
    ap.add_argument("--communicationTime", type=int, default=10, help="tau")
    ap.add_argument("--alpha", type=float, default=0.2)
    ap.add_argument("--deltaWire", default="fp32", choices=["fp32", "bf16"],
                    help="dtype of the client's delta push (bf16: half the bytes; every role must agree)")
    ap.add_argument("--testTime", type=int, default=100)
    ap.add_argument("--save", default="log")
    ap.add_argument("--resultsRoot", default="Results")
    ap.add_argument("--dataset", default="cifar10", choices=["cifar10", "mnist"])
    ap.add_argument("--trainSize", type=int, default=50000)
    ap.add_argument("--testSize", type=int, default=10000)
    ap.add_argument("--cuda", action="store_true")
    ap.add_argument("--backend", default="auto", choices=["auto", "hip", "torch"],
                    help="auto = the hand-written HIP executor for CIFAR-10 on a GPU, PyTorch ops otherwise")
    ap.add_argument("--graph", type=int, default=1, help="hipGraph capture of the client's steps (GPU)")
    ap.add_argument("--gpu", type=int, default=None)
    ap.add_argument("--commBackend", default="auto", choices=["auto", "rccl", "gloo"],
                    help="data plane (auto: RCCL on GPUs); gloo lets several roles share one GPU")
    ap.add_argument("--host", default=os.environ.get("MASTER_ADDR", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("MASTER_PORT", "8080")))
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--resume", action="store_true",
                    help="server: start from the center in Results/<save> (written by the tester)")
    ap.add_argument("--dieAfter", default=None, help=argparse.SUPPRESS)  # "client:syncs" fault injection (tests)
    ap.add_argument("--commTimeout", type=float, default=None,
                    help="seconds before a dead/stuck peer stops the run (default 600)")
    return ap.parse_args()


def main():
    opt = parse()
    if opt.commTimeout is not None:
        os.environ["DISTLEARN_COMM_TIMEOUT"] = str(opt.commTimeout)
    try:
        run(opt)
    except CommError as e:
        # a dead or stuck peer (reference: every role waited forever)
        print(f"easgd: communication failure: {e}", file=sys.stderr, flush=True)
        sys.exit(2)


def run(opt):
    N = opt.numNodes
    world = N + (1 if opt.noTester else 2)
    if opt.server:
        rank = 0
    elif opt.tester:
        rank = N + 1
    elif opt.role == "auto" and "RANK" in os.environ:
        rank = int(os.environ["RANK"])
    elif opt.role == "server":
        rank = 0
    elif opt.role == "tester":
        rank = N + 1
    else:
        rank = opt.nodeIndex
    role = "server" if rank == 0 else ("tester" if rank == N + 1 else "client")
    if opt.gpu is None:
        opt.gpu = rank + 1
    dev = device_of(opt)
    set_verbose(opt.verbose)
    tree = Tree(rank + 1, world, host=opt.host, port=opt.port, device=dev, backend=opt.commBackend)

    torch.manual_seed(0)
    model = (CifarConvNet(seed=0) if opt.dataset == "cifar10" else MnistConvNet(seed=0)).to(dev)
    ea = AsyncEA(tree, None, None, None, None, None, N, rank, opt.communicationTime, opt.alpha,
                 delta_wire=opt.deltaWire)
    cd = torch.bfloat16 if dev.type == "cuda" else torch.float32
    hip = opt.backend == "hip" or (opt.backend == "auto" and dev.type == "cuda" and opt.dataset == "cifar10")
    if hip and (dev.type != "cuda" or opt.dataset != "cifar10"):
        raise SystemExit("easgd: --backend hip needs --cuda and the CIFAR-10 convnet")

    if role == "server":
        flat = FlatParams(model, grads=False, shadow_bf16=False)
        if opt.resume:
            st = load_checkpoint(results_dir(opt.save, opt.resultsRoot), model)  # Net = the last tested center
            ea.syncs = int(st.get("server_syncs", 0))
            print(f"server: resumed center of snapshot {st.get('snapshot')} ({ea.syncs} syncs)")
        ea.initServer(flat)
        while ea.syncServer(flat):
            if ea.syncs % opt.testTime == 0:
                ea.testNet()
        ea.shutdown()
        print(f"server: {ea.syncs} syncs")
    elif role == "client":
        import time

        ds = Dataset(opt.dataset, rank, N, train=True, synthetic_size=opt.trainSize, device=dev)
        # grads -> syncClient (elastic move) -> SGD with the pre-move grads, every
        # step (EASGD_client.lua:97-119): DataParallelTrainer(algo="async") does
        # exactly that, on the HIP executor with unrolled hipGraphs on a GPU
        tr = DataParallelTrainer(model, tree, lr=opt.learningRate, algo="async", tau=opt.communicationTime,
                                 alpha=opt.alpha, backend="hip" if hip else "torch", compute_dtype=cd,
                                 graph=bool(opt.graph) and dev.type == "cuda", max_batch=opt.batchSize, async_ea=ea)
        fast = hip and tr.graph
        b = (DeviceLoader(ds, "permutation", opt.batchSize, seed=rank) if fast
             else ds.sampledBatcher("permutation", opt.batchSize, dtype=cd, seed=rank))
        tr.synchronize_parameters()  # initClient: receive the server's center
        die = [int(v) for v in opt.dieAfter.split(":")] if opt.dieAfter else None
        loss, steps, t0 = None, 0, time.perf_counter()
        for _ in range(opt.numEpochs):
            nb = b.numBatches() if not opt.maxSteps else min(opt.maxSteps, b.numBatches())
            done = 0
            while done < nb:
                # a syncing step at most every tau steps: run up to the next one
                k = min(nb - done, opt.communicationTime - ea.step % opt.communicationTime) if fast else 1
                loss = tr.run(b, k) if fast else tr.step(*b.getBatch())
                done += k
                if die and [rank, ea.syncs] == die:
                    os._exit(3)  # fault injection: this client dies without saying BYE
            steps += done
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        tr.finish()  # BYE
        print(f"client {rank}: {ea.syncs} syncs, {steps} steps, {steps * opt.batchSize / max(dt, 1e-9):.1f} img/s, "
              f"last loss {float(loss.detach()):.4f}")
    else:
        out = results_dir(opt.save, opt.resultsRoot)
        err_log = Logger(os.path.join(out, "ErrorRate.log"), ["Training Error", "Test Error"])
        txt = open(os.path.join(out, "Log.txt"), "a")
        txt.write(" ".join(sys.argv) + "\n")
        trd = Dataset(opt.dataset, 1, 1, train=True, synthetic_size=min(opt.trainSize, 2048), device=dev)
        te = Dataset(opt.dataset, 1, 1, train=False, synthetic_size=min(opt.testSize, 2048), device=dev)
        flat = FlatParams(model, grads=True, shadow_bf16=hip)
        # the reference tester evaluates the snapshot with its training-mode
        # functional model (batch statistics, EASGD_tester.lua:109-159)
        ex = make_executor(model, flat, max_batch=256) if hip else None
        ea.initTester(flat)
        n = 0
        while ea.startTest(flat):
            errs = []
            for ds in (trd, te):
                conf = ConfusionMatrix(10, device=dev)
                b = ds.sampledBatcher("linear", 256, dtype=cd)
                for _ in range(b.numBatches()):
                    x, y = b.getBatch()
                    conf.add(ex.predict(x, batch_stats=True) if ex is not None
                             else predict_module(model, x, cd, batch_stats=True), y)
                errs.append(1.0 - conf.totalValid)
            err_log.add({"Training Error": errs[0], "Test Error": errs[1]})
            txt.write(f"snapshot {n}: train error {errs[0]:.4f} test error {errs[1]:.4f}\n")
            txt.flush()
            n += 1
            # Net = the evaluated center (reference layout); optState = its counters
            save_checkpoint(out, model, {"center": ea.center, "snapshot": n, "server_syncs": ea.server_syncs,
                                         "lr": opt.learningRate, "tau": opt.communicationTime, "alpha": opt.alpha,
                                         "train_error": errs[0], "test_error": errs[1]})
            ea.finishTest()
        print(f"tester: {n} snapshots")
    tree.comm.barrier()


if __name__ == "__main__":
    main()
