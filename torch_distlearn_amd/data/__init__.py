"""Partitioned datasets and samplers (replaces torch-dataset).

Reference usage: ``Dataset(url, {partition = nodeIndex, partitions = numNodes})``
then ``:sampledBatcher{samplerKind = 'permutation' | 'label-uniform' |
'linear', batchSize, inputDims, processor}`` returning ``getBatch`` /
``numBatches`` closures (examples/mnist.lua:26-40, examples/cifar10.lua:41-92,
examples/Data.lua:10-61; SURVEY §2.4 "torch-dataset").

MI355X design (not a translation of the Lua worker threads):

* a node's whole partition lives in HBM as uint8 NHWC (CIFAR-10's 50k train
  images are 150 MB: nothing compared with 288 GB), so a step moves only the
  B sampled indices host->device;
* the index stream comes from the native C++ :class:`PartitionSampler`
  (csrc/runtime/loader.h: deterministic xoshiro streams per partition,
  ``linear`` / ``permutation`` / ``label-uniform`` / ``uniform``);
* the gather + ``(x/255 - mean)/std`` + cast to bf16 (+ channel zero-pad for
  the MFMA kernels) is ONE HIP kernel (csrc/kernels/metrics.hip
  ``gather_normalize``), so the "processor" callbacks of the reference run on
  the GPU;
* on CPU (gloo tests) the same sampler feeds plain torch indexing.

No dataset is downloaded (there is no network): :func:`load_cifar10` /
:func:`load_mnist` read the standard binary files if they are present
locally, and :func:`synthetic_cifar10` / :func:`synthetic_mnist` build
deterministic data of the same shapes.
"""
from __future__ import annotations

import os
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from .._native import available, native, stream_handle

SAMPLERS = {"linear": 0, "permutation": 1, "label-uniform": 2, "uniform": 3}

CIFAR_MEAN = (0.4914, 0.4822, 0.4465)
CIFAR_STD = (0.2470, 0.2435, 0.2616)
MNIST_MEAN = (0.1307, 0.0, 0.0)
MNIST_STD = (0.3081, 1.0, 1.0)


# ---------------------------------------------------------------------------
# python sampler (same semantics as the native one; used when _C is absent)
# ---------------------------------------------------------------------------
class _PySampler:
    def __init__(self, n, labels, num_classes, partition, partitions, kind, seed):
        self.lo = n * partition // partitions
        self.hi = n * (partition + 1) // partitions
        self.kind = kind
        self.rng = np.random.default_rng(seed * 1000003 + partition)
        if kind == SAMPLERS["label-uniform"]:
            lab = np.asarray(labels[self.lo:self.hi])
            self.by_class = [np.nonzero(lab == c)[0] + self.lo for c in range(num_classes)]
            self.by_class = [v for v in self.by_class if len(v)]
        self.reset_epoch()

    def size(self):
        return self.hi - self.lo

    def num_batches(self, b):
        return (self.size() + b - 1) // b

    def reset_epoch(self):
        self.pos = 0
        if self.kind == SAMPLERS["permutation"]:
            self.perm = self.rng.permutation(self.size()) + self.lo

    def next_batch_np(self, batch):
        out = np.empty(batch, dtype=np.int64)
        valid = batch
        for b in range(batch):
            if self.kind in (0, 1):
                if self.pos >= self.size():
                    if b > 0:
                        valid = min(valid, b)
                        out[b] = out[b - 1]
                        continue
                    self.reset_epoch()
                out[b] = self.lo + self.pos if self.kind == 0 else self.perm[self.pos]
                self.pos += 1
            elif self.kind == 2:
                cls = self.by_class[self.rng.integers(len(self.by_class))]
                out[b] = cls[self.rng.integers(len(cls))]
            else:
                out[b] = self.lo + self.rng.integers(self.size())
        return out, valid


def make_sampler(n: int, labels: Optional[Sequence[int]], num_classes: int, partition: int, partitions: int,
                 kind: str, seed: int = 0):
    """``partition`` is 1-based like the reference's ``nodeIndex``."""
    k = SAMPLERS[kind]
    p0 = int(partition) - 1
    lab = [] if labels is None else [int(v) for v in labels]
    if available():
        return native().PartitionSampler(int(n), lab, int(num_classes), p0, int(partitions), k, int(seed))
    return _PySampler(n, lab, num_classes, p0, partitions, k, seed)


def _next_indices(sampler, batch: int, buf: torch.Tensor) -> int:
    if isinstance(sampler, _PySampler):
        idx, valid = sampler.next_batch_np(batch)
        buf[:batch].copy_(torch.from_numpy(idx))
        return int(valid)
    return int(sampler.next_batch(buf.data_ptr(), batch))


# ---------------------------------------------------------------------------
# dataset + batcher
# ---------------------------------------------------------------------------
class PartitionedDataset:
    """A node's view of a dataset: uint8 images [N, H, W, C] + int64 labels."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, partition: int = 1, partitions: int = 1,
                 num_classes: int = 10, mean=CIFAR_MEAN, std=CIFAR_STD, device=None):
        if images.dtype != torch.uint8 or images.dim() != 4:
            raise ValueError("images must be uint8 [N, H, W, C]")
        self.partition, self.partitions = int(partition), int(partitions)
        self.num_classes = num_classes
        self.mean, self.std = tuple(mean), tuple(std)
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        # the whole dataset is resident on the device (HBM); the sampler picks this
        # node's partition (partition slices are contiguous like torch-dataset's)
        self.images = images.to(self.device).contiguous()
        self.labels = labels.to(torch.int64).to(self.device).contiguous()
        self.labels_host = labels.to(torch.int64).cpu()
        self.N, self.H, self.W, self.C = self.images.shape

    def sampledBatcher(self, samplerKind: str = "permutation", batchSize: int = 32, channels_out: Optional[int] = None,  # noqa: N802,N803
                       dtype=torch.bfloat16, seed: int = 0) -> "Batcher":
        return Batcher(self, samplerKind, batchSize, channels_out or self.C, dtype, seed)

    sampled_batcher = sampledBatcher

    def size(self) -> int:
        return self.N * (self.partition) // self.partitions - self.N * (self.partition - 1) // self.partitions


class Batcher:
    """``getBatch()`` -> (x NHWC normalised, y int64), ``numBatches()``."""

    def __init__(self, ds: PartitionedDataset, kind: str, batch: int, channels_out: int, dtype, seed: int):
        self.ds, self.batch, self.cout, self.dtype = ds, int(batch), int(channels_out), dtype
        self.sampler = make_sampler(ds.N, ds.labels_host.tolist() if kind == "label-uniform" else None,
                                    ds.num_classes, ds.partition, ds.partitions, kind, seed)
        self.idx_host = torch.empty(self.batch, dtype=torch.int64).pin_memory() if ds.device.type == "cuda" \
            else torch.empty(self.batch, dtype=torch.int64)
        self.idx_dev = torch.empty(self.batch, dtype=torch.int64, device=ds.device)
        self.out = torch.empty(self.batch, ds.H, ds.W, self.cout, dtype=dtype, device=ds.device)
        self.valid = self.batch
        self.drawn = 0  # batches drawn so far (checkpointed so a resumed run continues the stream)

    def numBatches(self) -> int:  # noqa: N802
        return int(self.sampler.num_batches(self.batch))

    num_batches = numBatches

    def reset(self) -> None:
        self.sampler.reset_epoch()

    def skip(self, nbatches: int) -> None:
        """Advance the sample stream by ``nbatches`` batches without gathering
        them (resume: continue exactly where the checkpointed run was)."""
        for _ in range(int(nbatches)):
            _next_indices(self.sampler, self.batch, self.idx_host)
        self.drawn += int(nbatches)

    def getBatch(self) -> Tuple[torch.Tensor, torch.Tensor]:  # noqa: N802
        self.drawn += 1
        self.valid = _next_indices(self.sampler, self.batch, self.idx_host)
        ds = self.ds
        if ds.device.type == "cuda":
            self.idx_dev.copy_(self.idx_host, non_blocking=True)
            if self.dtype != torch.bfloat16:
                raise ValueError("device batcher produces bf16")
            m, s = (list(ds.mean) + [0.0] * 3)[:3], (list(ds.std) + [1.0] * 3)[:3]
            native().gather_normalize(ds.images.data_ptr(), self.idx_dev.data_ptr(), self.out.data_ptr(), self.batch,
                                      ds.H * ds.W, ds.C, self.cout, m[0], m[1], m[2], s[0], s[1], s[2],
                                      stream_handle())
            y = ds.labels.index_select(0, self.idx_dev)
            return self.out, y
        idx = self.idx_host
        x = ds.images.index_select(0, idx).float().div_(255.0)
        mean = torch.tensor(ds.mean[:ds.C], dtype=torch.float32)
        std = torch.tensor(ds.std[:ds.C], dtype=torch.float32)
        x = (x - mean) / std
        if self.cout > ds.C:
            x = torch.nn.functional.pad(x, (0, self.cout - ds.C))
        return x.to(self.dtype), ds.labels.index_select(0, idx)

    get_batch = getBatch


class DeviceLoader:
    """Device-side batching for graph-captured training steps.

    The sample order (from the same native sampler as :class:`Batcher`) lives
    in HBM as an int32 ring of TWO epochs; a step's batch is selected by a
    device-resident step counter -- step s reads ``order[(s*B + b) mod 2n]`` --
    and gathered + normalised + padded by the native executor's first kernel
    (``prep_step_gather``); a later kernel of the same step advances the
    counter.  A captured hipGraph therefore replays consecutive batches with
    no per-step host work and no host->device copies, across an epoch
    boundary too.  :meth:`step_done` keeps the host's count; when an epoch is
    used up the host generates the order two epochs ahead into a pinned
    buffer and uploads it, asynchronously and stream-ordered behind the steps
    already queued, into the half the finished epoch occupied -- no pageable
    copy, no host stall inside the training loop (at N=8
    an epoch is 48 steps, so every timed window used to contain one).

    Paths without the native executor call :meth:`getBatch` (eager gather of
    the same batch sequence).
    """

    def __init__(self, ds: PartitionedDataset, kind: str = "permutation", batch: int = 32, seed: int = 0):
        self.ds, self.batch = ds, int(batch)
        self.H, self.W = ds.H, ds.W
        self.sampler = make_sampler(ds.N, ds.labels_host.tolist() if kind == "label-uniform" else None,
                                    ds.num_classes, ds.partition, ds.partitions, kind, seed)
        self.steps_per_epoch = max(1, int(self.sampler.size()) // self.batch)
        n = self.steps_per_epoch * self.batch
        self.order = torch.empty(2 * n, dtype=torch.int32, device=ds.device)  # epochs e, e+1 (halves e % 2)
        self.ctr = torch.zeros(2, dtype=torch.int64, device=ds.device)  # [step, reserved]
        self.labels_out = torch.empty(self.batch, dtype=torch.int64, device=ds.device)
        self._host_steps = 0
        self.epoch = 0
        self._idx = torch.empty(self.batch, dtype=torch.int64)
        cuda = self.order.is_cuda
        self._pinned = [torch.empty(n, dtype=torch.int32, pin_memory=cuda) for _ in range(2)]
        self._upload_ev = [None, None]
        self._upload(0)
        self._upload(1)

    def _upload(self, half: int) -> None:
        """Generate the sampler's next epoch and upload it into ``half`` of the
        ring (stream-ordered on the current stream)."""
        self.sampler.reset_epoch()
        rows = []
        for _ in range(self.steps_per_epoch):
            _next_indices(self.sampler, self.batch, self._idx)
            rows.append(self._idx.clone())
        n = self.steps_per_epoch * self.batch
        src = self._pinned[half]
        ev = self._upload_ev[half]
        if ev is not None:
            ev.synchronize()  # this pinned buffer's previous upload (an epoch ago) has run
        src.copy_(torch.cat(rows))
        self.order[half * n:(half + 1) * n].copy_(src, non_blocking=True)
        if self.order.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
            self._upload_ev[half] = ev

    def _next_epoch(self) -> None:
        # the finished epoch's half takes the epoch after the next one
        self._upload(self.epoch % 2)
        self.epoch += 1
        self._host_steps = 0

    def numBatches(self) -> int:  # noqa: N802
        return self.steps_per_epoch

    num_batches = numBatches

    @property
    def drawn(self) -> int:
        """Batches consumed so far (checkpointed: a resumed run continues the stream)."""
        return self.epoch * self.steps_per_epoch + self._host_steps

    def skip(self, nbatches: int) -> None:
        """Advance the sample stream by ``nbatches`` batches (resume)."""
        n = int(nbatches)
        while n >= self.steps_per_epoch - self._host_steps:
            n -= self.steps_per_epoch - self._host_steps
            self._next_epoch()
        self._host_steps += n
        self.ctr[0] = (self.epoch % 2) * self.steps_per_epoch + self._host_steps

    def gather_args(self):
        ds = self.ds
        return (ds.images.data_ptr(), self.order.data_ptr(), ds.labels.data_ptr(), self.labels_out.data_ptr(),
                self.ctr.data_ptr(), int(self.order.numel()), ds.C, [float(v) for v in ds.mean[:ds.C]],
                [float(v) for v in ds.std[:ds.C]])

    def step_done(self) -> None:
        """Host bookkeeping after a step consumed a batch: once an epoch is
        used up, refill its half of the ring (the device counter runs on into
        the next half, already uploaded)."""
        self._host_steps += 1
        if self._host_steps >= self.steps_per_epoch:
            self._next_epoch()

    def getBatch(self) -> Tuple[torch.Tensor, torch.Tensor]:  # noqa: N802
        """Eager equivalent (the same batch the device path would use):
        (x NHWC normalised, y int64); advances the counter."""
        k = int(self.ctr[0].item()) % (2 * self.steps_per_epoch)
        idx = self.order[k * self.batch:(k + 1) * self.batch].to(torch.int64)
        ds = self.ds
        x = ds.images.index_select(0, idx).float().div_(255.0)
        mean = torch.tensor(ds.mean[:ds.C], dtype=torch.float32, device=x.device)
        std = torch.tensor(ds.std[:ds.C], dtype=torch.float32, device=x.device)
        x = ((x - mean) / std)
        self.ctr[0] += 1
        y = ds.labels.index_select(0, idx)
        self.labels_out.copy_(y)
        return x, y

    get_batch = getBatch


# ---------------------------------------------------------------------------
# sources
# ---------------------------------------------------------------------------
def synthetic_images(n: int, hw: int, c: int, num_classes: int = 10, seed: int = 0):
    """Deterministic class-dependent uint8 images (learnable, not pure noise).
    The class prototypes do not depend on ``seed`` (only labels and noise
    do), so a train split and a test split drawn with different seeds share
    their classes and test accuracy measures generalisation."""
    g = torch.Generator().manual_seed(seed)
    labels = torch.randint(0, num_classes, (n,), generator=g)
    gp = torch.Generator().manual_seed(0x5EED0 + num_classes * 1000 + hw * 10 + c)
    proto = torch.randint(0, 256, (num_classes, hw, hw, c), generator=gp, dtype=torch.int32)
    noise = torch.randint(-48, 49, (n, hw, hw, c), generator=g, dtype=torch.int32)
    imgs = (proto[labels] + noise).clamp_(0, 255).to(torch.uint8)
    return imgs, labels


def synthetic_cifar10(n: int = 50000, seed: int = 0):
    return synthetic_images(n, 32, 3, 10, seed)


def synthetic_mnist(n: int = 60000, seed: int = 0, hw: int = 32):
    """MNIST-shaped (the reference reshapes 1024-dim inputs to 1x32x32, examples/mnist.lua:34,53)."""
    return synthetic_images(n, hw, 1, 10, seed)


def load_cifar10(root: str, train: bool = True):
    """Read the CIFAR-10 binary release (data_batch_*.bin / test_batch.bin) from
    ``root`` if present; returns (uint8 NHWC images, int64 labels) or None."""
    names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
    paths = [os.path.join(root, n) for n in names]
    if not all(os.path.exists(p) for p in paths):
        return None
    raw = np.concatenate([np.fromfile(p, dtype=np.uint8).reshape(-1, 3073) for p in paths])
    labels = torch.from_numpy(raw[:, 0].astype(np.int64))
    imgs = torch.from_numpy(raw[:, 1:].reshape(-1, 3, 32, 32).transpose(0, 2, 3, 1).copy())
    return imgs, labels


def load_mnist(root: str, train: bool = True, pad_to: int = 32):
    """Read MNIST idx files from ``root`` if present (zero-padded 28->32 like
    the reference's 1024-dim inputs)."""
    pre = "train" if train else "t10k"
    ip = os.path.join(root, f"{pre}-images-idx3-ubyte")
    lp = os.path.join(root, f"{pre}-labels-idx1-ubyte")
    if not (os.path.exists(ip) and os.path.exists(lp)):
        return None
    imgs = np.fromfile(ip, dtype=np.uint8)[16:].reshape(-1, 28, 28)
    labels = np.fromfile(lp, dtype=np.uint8)[8:].astype(np.int64)
    p = (pad_to - 28) // 2
    imgs = np.pad(imgs, ((0, 0), (p, pad_to - 28 - p), (p, pad_to - 28 - p)))[..., None]
    return torch.from_numpy(imgs.copy()), torch.from_numpy(labels)


def Dataset(name: str = "cifar10", partition: int = 1, partitions: int = 1, train: bool = True,  # noqa: N802
            root: Optional[str] = None, synthetic_size: Optional[int] = None, device=None) -> PartitionedDataset:
    """Reference-style constructor: local files under ``root`` if present,
    otherwise synthetic data of the same shape."""
    name = name.lower()
    if name.startswith("cifar"):
        src = load_cifar10(root, train) if root else None
        if src is None:
            src = synthetic_cifar10(synthetic_size or (50000 if train else 10000), seed=0 if train else 1)
        return PartitionedDataset(*src, partition=partition, partitions=partitions, mean=CIFAR_MEAN, std=CIFAR_STD,
                                  device=device)
    if name.startswith("mnist"):
        src = load_mnist(root, train) if root else None
        if src is None:
            src = synthetic_mnist(synthetic_size or (60000 if train else 10000), seed=0 if train else 1)
        return PartitionedDataset(*src, partition=partition, partitions=partitions, mean=MNIST_MEAN[:1],
                                  std=MNIST_STD[:1], device=device)
    raise ValueError(f"unknown dataset {name!r}")


__all__ = ["Dataset", "PartitionedDataset", "Batcher", "make_sampler", "synthetic_cifar10", "synthetic_mnist",
           "load_cifar10", "load_mnist", "SAMPLERS"]
