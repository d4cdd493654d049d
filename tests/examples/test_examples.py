"""Example smoke tests: the reference's example programs,
run through the launcher on CPU/gloo with tiny synthetic datasets."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _launch(nproc, script, *args, extra=(), timeout=300, cwd=None):
    cmd = [sys.executable, "-m", "torch_distlearn_amd.launch", "--nproc", str(nproc), *extra,
           os.path.join(ROOT, "examples", script), *args]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=cwd or ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_mnist_allreduce_sgd_uneven_partitions():
    # 200 samples over 3 nodes -> partitions of 66/67/67: different step counts per node,
    # reconciled by the drain protocol of synchronizeParameters
    out = _launch(3, "mnist.py", "--epochs", "2", "--trainSize", "200", "--batchSize", "4")
    assert "Epoch 2" in out and "global correct" in out


def test_mnist_mlp_baseline_config1():
    out = _launch(2, "mnist.py", "--model", "mlp", "--epochs", "1", "--trainSize", "256", "--batchSize", "8")
    assert "Epoch 1" in out


def test_mnist_allreduce_ea():
    out = _launch(2, "mnist_ea.py", "--epochs", "2", "--trainSize", "200", "--batchSize", "4", "--tau", "3")
    assert "Epoch 2" in out


def test_cifar10_two_nodes():
    out = _launch(2, "cifar10.py", "--epochs", "1", "--maxSteps", "3", "--batchSize", "8", "--trainSize", "256",
                  "--testSize", "64", "--learningRate", "0.01")
    assert "test accuracy" in out


def test_cifar10_two_nodes_reaches_test_accuracy():
    """The reference example's purpose is the all-reduced test confusion
    matrix (examples/cifar10.lua:213-236): on the synthetic CIFAR-shaped data
    (class prototypes + noise, shared by the train and test splits) one epoch
    of 64 steps per node must classify the held-out split (>= 95 %)."""
    import re

    out = _launch(2, "cifar10.py", "--epochs", "1", "--batchSize", "64", "--trainSize", "4096", "--testSize", "256",
                  timeout=600)
    acc = [float(m) for m in re.findall(r"test accuracy ([0-9.]+)%", out)]
    assert acc and acc[-1] >= 95.0, out[-2000:]


def test_async_easgd_roles(tmp_path):
    out = _launch(4, "easgd.py", "--numNodes", "2", "--dataset", "mnist", "--trainSize", "256", "--batchSize", "16",
                  "--communicationTime", "2", "--testTime", "2", "--numEpochs", "1",
                  "--resultsRoot", str(tmp_path / "Results"), extra=("--no-node-flags",))
    assert "server:" in out and "tester:" in out
    d = tmp_path / "Results" / "log"
    assert (d / "ErrorRate.log").read_text().splitlines()[0] == "Training Error\tTest Error"
    assert (d / "Net").exists() and (d / "optState").exists()
    import torch

    st = torch.load(d / "optState", weights_only=True)
    net = torch.load(d / "Net", weights_only=True)
    # the tester's checkpoint is the evaluated center (Net, reference layout) plus its counters
    assert st["snapshot"] >= 1 and st["server_syncs"] >= 2 and st["tau"] == 2
    flat_center = st["center"]
    assert torch.equal(flat_center[64:64 + net[0].numel()], net[0].reshape(-1))
    # the server restarts from that center (--resume)
    out = _launch(4, "easgd.py", "--numNodes", "2", "--dataset", "mnist", "--trainSize", "64", "--batchSize", "16",
                  "--communicationTime", "2", "--testTime", "2", "--numEpochs", "1", "--resume",
                  "--resultsRoot", str(tmp_path / "Results"), extra=("--no-node-flags",))
    assert f"resumed center of snapshot {st['snapshot']}" in out


def test_async_easgd_dead_client_exits_nonzero(tmp_path):
    """examples/easgd.py with a client that dies: the server and tester exit
    non-zero with a communication error within --commTimeout (no hang)."""
    cmd = [sys.executable, "-m", "torch_distlearn_amd.launch", "--nproc", "4", "--no-node-flags",
           os.path.join(ROOT, "examples", "easgd.py"), "--numNodes", "2", "--dataset", "mnist", "--trainSize", "4096",
           "--batchSize", "16", "--communicationTime", "2", "--testTime", "2", "--numEpochs", "20",
           "--commTimeout", "5", "--dieAfter", "2:3", "--resultsRoot", str(tmp_path / "Results")]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "communication failure" in r.stderr and "clients [2]" in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("algo", ["sgd", "ea", "async"])
def test_bench_contract_cpu(algo):
    """bench.py under torch.distributed.run (the driver's N>1 launch), run on
    CPU/gloo: one JSON line from rank 0 with whole-job images/s; AsyncEA = rank 0
    parameter server + 2 clients (BASELINE configs 2-4 plumbing)."""
    import json
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "3", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "3",
           "--warmup", "1", "--device", "cpu", "--batch", "4", "--algo", algo, "--tau", "2"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 3 and out["steps"] == 3 and out["warmup"] == 1 and out["higher_is_better"]
    workers = 2 if algo == "async" else 3
    assert out["config"]["global_batch"] == 4 * workers
    # (value is rounded to 0.1 img/s: at CPU speed that alone can exceed 1e-3 relative)
    assert abs(out["value"] - 4 * workers * 1000.0 / out["ms_per_step"]) <= max(1e-3 * out["value"], 0.051)


def test_bench_self_launch_cpu():
    """``python3 bench.py --gpus 4`` as a plain command (the driver's BENCH
    command shape): bench.py spawns its own 4 ranks and prints ONE JSON line."""
    import json

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--device", "cpu", "--gpus", "4", "--steps", "3",
           "--warmup", "1", "--batch", "4"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 4 and out["config"]["parallelism"] == "dp4" and out["config"]["global_batch"] == 16
    assert out["config"]["grad_comm_dtype"] == "fp32" and "device_ids" in out["config"]


def test_bench_self_launch_fails_fast_without_gpus():
    """``--gpus 2`` on a box with fewer GPUs: every rank exits with a clear
    message before any rendezvous and the launcher returns non-zero at once."""
    import time

    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1"]
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env.pop("WORLD_SIZE", None)
    t0 = time.time()
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and time.time() - t0 < 90
    assert "needs 2 GPUs" in r.stderr, r.stderr[-2000:]
    assert r.stdout.strip() == ""


def test_allreduce_bw_script_gloo():
    # scripts/allreduce_bw.py (data-plane bandwidth sweep) on 2 gloo ranks
    import json

    from torch_distlearn_amd.launch import free_port

    cmd = [sys.executable, "-m", "torch.distributed.run", "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
           "--master-port", str(free_port()), os.path.join(ROOT, "scripts", "allreduce_bw.py"), "--device", "cpu",
           "--max-mb", "1", "--iters", "2", "--warmup", "1"]
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rows = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [x["bytes"] for x in rows] == [65536, 262144, 1048576]
    assert all(x["n_ranks"] == 2 and x["busbw_GBps"] > 0 for x in rows)
