"""DeviceLoader's two-epoch order ring (CPU tensors; the GPU tests in
tests/kernels/test_engine_gpu.py drive the same ring through the gather kernel):
the batch stream equals the sampler's own epoch-by-epoch stream, the device
counter runs on across epoch boundaries, and a resumed loader (skip) continues
the stream exactly."""
import torch

from torch_distlearn_amd.data import DeviceLoader, PartitionedDataset, _next_indices, make_sampler, synthetic_cifar10


def _ds(partition=1, partitions=2):
    imgs, labels = synthetic_cifar10(200, seed=3)
    return PartitionedDataset(imgs, labels, partition, partitions)


def _sampler_stream(ds, kind, batch, nbatches, seed=0):
    """Reference: epoch orders drawn from a fresh sampler, one epoch at a time."""
    s = make_sampler(ds.N, ds.labels_host.tolist() if kind == "label-uniform" else None, ds.num_classes,
                     ds.partition, ds.partitions, kind, seed)
    spe = max(1, int(s.size()) // batch)
    buf = torch.empty(batch, dtype=torch.int64)
    out = []
    while len(out) < nbatches:
        s.reset_epoch()
        for _ in range(spe):
            _next_indices(s, batch, buf)
            out.append(buf.clone())
    return out[:nbatches]


def _drain(ld, n):
    ys = []
    for _ in range(n):
        _, y = ld.getBatch()
        ys.append(y.clone())
        ld.step_done()
    return ys


def test_stream_matches_sampler_across_epochs():
    for kind in ("permutation", "label-uniform"):
        ds = _ds()
        ld = DeviceLoader(ds, kind=kind, batch=16)
        assert ld.steps_per_epoch == 6 and ld.order.numel() == 2 * 6 * 16
        n = 5 * ld.steps_per_epoch + 3
        ys = _drain(ld, n)
        ref = _sampler_stream(ds, kind, 16, n)
        for y, idx in zip(ys, ref):
            assert torch.equal(y, ds.labels.index_select(0, idx))
        assert ld.epoch == 5 and ld._host_steps == 3
        assert int(ld.ctr[0]) == n  # the device counter never resets; the gather wraps mod 2 epochs


def test_skip_resumes_the_stream():
    ds = _ds(2, 2)
    a = DeviceLoader(ds, batch=16, seed=7)
    ya = _drain(a, 20)
    for k in (0, 5, 6, 13):
        b = DeviceLoader(ds, batch=16, seed=7)
        b.skip(k)
        assert b.drawn == k
        yb = _drain(b, 20 - k)
        assert all(torch.equal(u, v) for u, v in zip(ya[k:], yb))
