"""End-to-end checkpoint / resume (the reference declares
Results/<save>/{Net, optState} in examples/EASGD_tester.lua:36-47 but never
writes or reads them).

2 gloo nodes train the MNIST convnet example (uneven partitions, so the
epoch-end drain runs) for 2 epochs straight; a second job trains 1 epoch with
``--save``, and a third, fresh job ``--resume``s it and trains epoch 2.  The
final parameters must be BITWISE those of the uninterrupted run for
AllReduceSGD, and for AllReduceEA (every node's own elastic replica and the
center are restored)."""
import os
import sys

import pytest

from tests import mp

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, port, algo, root, epochs, save, resume):
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import mnist  # examples/mnist.py

    args = ["--nodeIndex", str(rank + 1), "--numNodes", str(world), "--port", str(port), "--epochs", str(epochs),
            "--trainSize", "70", "--batchSize", "4", "--learningRate", "0.05", "--resultsRoot", root]
    if save:
        args += ["--save", "ckpt"]
    if resume:
        args += ["--resume"]
    ap = mnist.parser("resume test")
    if algo == "ea":
        ap.add_argument("--tau", type=int, default=3)
        ap.add_argument("--alpha", type=float, default=0.3)
    tr = mnist.run(ap.parse_args(args), algo)
    out = {"p": tr.flat.data.clone()}
    if tr.ea is not None:
        out["c"] = tr.ea.center.clone()
    return out


@pytest.mark.parametrize("algo", ["sgd", "ea"])
def test_resume_is_bitwise(algo, tmp_path):
    root = str(tmp_path)
    straight = mp.run(_worker, 2, algo, root, 2, False, False)
    mp.run(_worker, 2, algo, root, 1, True, False)
    assert os.path.exists(os.path.join(root, "ckpt", "Net"))
    assert os.path.exists(os.path.join(root, "ckpt", "optState"))
    resumed = mp.run(_worker, 2, algo, root, 2, True, True)
    for a, b in zip(straight, resumed):
        assert a["p"].tobytes() == b["p"].tobytes()
        if "c" in a:
            assert a["c"].tobytes() == b["c"].tobytes()
    if algo == "sgd":
        assert straight[0]["p"].tobytes() == straight[1]["p"].tobytes()
