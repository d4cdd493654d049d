"""Partitioned samplers / datasets (replacement of torch-dataset)."""
import torch

from torch_distlearn_amd.data import Dataset, PartitionedDataset, _PySampler, make_sampler, synthetic_cifar10


def _draw(s, batch, n):
    buf = torch.empty(batch, dtype=torch.int64)
    out = []
    for _ in range(n):
        v = s.next_batch(buf.data_ptr(), batch) if not isinstance(s, _PySampler) else None
        if v is None:
            idx, v = s.next_batch_np(batch)
            buf.copy_(torch.from_numpy(idx))
        out.append((v, buf.clone()))
    return out


def test_partitions_cover_dataset_disjointly():
    N, P = 103, 4
    seen = []
    for p in range(1, P + 1):
        s = make_sampler(N, None, 10, p, P, "linear")
        n = s.size()
        got = [int(i) for v, b in _draw(s, n, 1) for i in b[:v]]
        seen += got
    assert sorted(seen) == list(range(N))


def test_permutation_epoch_is_a_permutation_and_changes():
    s = make_sampler(64, None, 10, 2, 2, "permutation", seed=3)
    e1 = torch.cat([b[:v] for v, b in _draw(s, 8, 4)])
    e2 = torch.cat([b[:v] for v, b in _draw(s, 8, 4)])
    assert sorted(e1.tolist()) == list(range(32, 64)) == sorted(e2.tolist())
    assert not torch.equal(e1, e2)


def test_short_last_batch_reports_valid_count():
    s = make_sampler(10, None, 10, 1, 1, "linear")
    (v1, _), (v2, b2) = _draw(s, 8, 2)
    assert v1 == 8 and v2 == 2 and b2[:2].tolist() == [8, 9]


def test_label_uniform_balances_classes():
    labels = [0] * 90 + [1] * 10
    s = make_sampler(100, labels, 2, 1, 1, "label-uniform", seed=1)
    draws = torch.cat([b for _, b in _draw(s, 100, 10)])
    frac1 = float((draws >= 90).float().mean())
    assert 0.4 < frac1 < 0.6


def test_native_and_python_samplers_agree_on_partition_ranges():
    for kind in ("linear", "permutation"):
        n = make_sampler(50, None, 10, 3, 4, kind)
        p = _PySampler(50, [], 10, 2, 4, {"linear": 0, "permutation": 1}[kind], 0)
        assert n.size() == p.size() == 50 * 3 // 4 - 50 * 2 // 4


def test_batcher_normalises_and_pads_channels():
    imgs, labels = synthetic_cifar10(64)
    ds = PartitionedDataset(imgs, labels, 1, 2)
    b = ds.sampledBatcher("linear", 8, channels_out=8, dtype=torch.float32)
    x, y = b.getBatch()
    assert x.shape == (8, 32, 32, 8) and not x[..., 3:].any()
    ref = (imgs[:8].float() / 255 - torch.tensor(ds.mean)) / torch.tensor(ds.std)
    torch.testing.assert_close(x[..., :3], ref)
    assert torch.equal(y, labels[:8])


def test_dataset_factory_synthetic_shapes():
    ds = Dataset("mnist", 1, 3, synthetic_size=30)
    assert ds.images.shape == (30, 32, 32, 1) and ds.size() == 10
