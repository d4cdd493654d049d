"""Checkpoint layout (Results/<save>/{Net, optState}) and metrics."""
import os

import torch

from torch_distlearn_amd.checkpoint import load_checkpoint, save_checkpoint
from torch_distlearn_amd.models import CifarConvNet, MnistConvNet
from torch_distlearn_amd.utils.metrics import ConfusionMatrix, JsonlMetrics, Logger


def test_cifar_net_checkpoint_reference_layout(tmp_path):
    m = CifarConvNet(seed=1)
    save_checkpoint(str(tmp_path), m, {"lr": 0.1, "stepsPerNode": torch.tensor([3, 4])})
    net = torch.load(os.path.join(tmp_path, "Net"), weights_only=True)
    # SpatialConvolutionMM layout [Cout, Cin*5*5] in (c, kh, kw) order
    assert [tuple(t.shape) for t in net[:4]] == [(64, 75), (64,), (64,), (64,)]
    assert torch.equal(net[0].reshape(64, 3, 5, 5), m.conv1_w.detach().permute(0, 3, 1, 2))
    assert tuple(net[-2].shape) == (10, 2048) and len(net) == 18
    m2 = CifarConvNet(seed=2)
    st = load_checkpoint(str(tmp_path), m2)
    assert st["lr"] == 0.1 and st["stepsPerNode"].tolist() == [3, 4]
    x = torch.randn(2, 32, 32, 3)
    m.eval()
    m2.eval()
    torch.testing.assert_close(m(x), m2(x))


def test_generic_table_checkpoint(tmp_path):
    params = {"w": torch.randn(3, 4), "b": torch.randn(4)}
    save_checkpoint(str(tmp_path), params)
    other = {"w": torch.zeros(3, 4), "b": torch.zeros(4)}
    load_checkpoint(str(tmp_path), other)
    assert torch.equal(other["w"], params["w"]) and torch.equal(other["b"], params["b"])


def test_mnist_checkpoint_roundtrip(tmp_path):
    m = MnistConvNet(seed=4)
    save_checkpoint(str(tmp_path), m)
    m2 = MnistConvNet(seed=5)
    load_checkpoint(str(tmp_path), m2)
    for a, b in zip(m.parameters(), m2.parameters()):
        assert torch.equal(a, b)


def test_confusion_matrix_cpu():
    cm = ConfusionMatrix(3)
    pred = torch.tensor([[0.9, 0.1, 0.0], [0.1, 0.8, 0.1], [0.7, 0.2, 0.1], [0.0, 0.1, 0.9]])
    cm.add(pred, torch.tensor([0, 1, 1, 2]))
    assert cm.mat.tolist() == [[1, 0, 0], [1, 1, 0], [0, 0, 1]]
    assert abs(cm.totalValid - 0.75) < 1e-9
    assert "global correct: 75.000%" in str(cm)


def test_logger_and_jsonl(tmp_path):
    lg = Logger(str(tmp_path / "ErrorRate.log"), ["Training Error", "Test Error"])
    lg.add({"Training Error": 0.5, "Test Error": 0.25})
    lg.close()
    lines = (tmp_path / "ErrorRate.log").read_text().splitlines()
    assert lines == ["Training Error\tTest Error", "5.0000e-01\t2.5000e-01"]
    j = JsonlMetrics(str(tmp_path / "m.jsonl"))
    j.log(step=1, loss=2.0)
    j.close()
    assert '"loss": 2.0' in (tmp_path / "m.jsonl").read_text()
