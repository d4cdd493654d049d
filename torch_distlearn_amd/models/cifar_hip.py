"""Native executor for the CIFAR-10 convnet: every forward/backward op is a
hand-written gfx950 HIP kernel (csrc/kernels/{conv_igemm,bn_pool,head}.hip),
launched on the current HIP stream with static workspaces, so the whole step
is hipGraph-capturable.

Reference computation: examples/cifar10.lua:146-169 (predict / f / df via
torch-autograd + cunn).  Per block i:

  forward   conv_fwd (MFMA implicit GEMM, epilogue: BN partial sums)
            bn_finalize (batch mean/invstd, running stats)
            bn_relu_pool_fwd
  head      head_fwd_bwd (Linear + LogSoftMax + NLL + dlogits + dh), head_wgrad
  backward  bn_relu_pool_bwd_reduce -> bn_bwd_finalize (dgamma, dbeta)
            -> bn_relu_pool_bwd_apply (dy) -> conv_wgrad (-> slab_reduce)
            -> conv dgrad (= conv_fwd on dy with flipped/transposed weights)

Side streams (the dgrad weight transposes during the forward, a block's
weight gradient beside its dgrad) were measured as net losses inside the
hipGraph (0.531 / 0.567 vs 0.480 ms/step, round 1) and removed in round 6:
every kernel of the step spans the 256 CUs and a cross-queue edge costs more
than the overlap wins.

Gradients are written (fp32) straight into the flat gradient buffer; as soon
as a block's gradients are final its leaves are reported to the
:class:`~torch_distlearn_amd.parallel.buckets.GradBucketer`, which launches
that bucket's RCCL all-reduce on the comm stream while the remaining blocks'
backward runs.  Weights are read as the bf16 shadow that the fused SGD kernel
refreshes (conv) or as the fp32 master (BN affine, classifier).
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch

from .._native import native, stream_handle
from ..ops.flat import HEADER
from ..parallel.comm import runs_collectives
from .cifar_convnet import BN_EPS, BN_MOMENTUM, KSIZE, CifarConvNet

BF16 = torch.bfloat16
CIN_PAD = 8  # the 3-channel input layer zero-padded to 8 channels (one 16-B vector per tap); the default
#              pair-packed layer 1 reads a 4-channel input instead (CifarHIPExecutor.kin0, pair1)
SPAD = KSIZE // 2  # spatial zero border of every convolution input (written once, never touched)

# tile ids of conv_fwd: 0 = 128x128, 1 = 64x64, 2 = 128x64 (BK = 64) ; conv_wgrad: 1 = 64x64, 2 = 128x128
_FWD_TILES = {0: (128, 128), 1: (64, 64), 2: (128, 64)}


def _fwd_plan(M: int, N: int, K: int, batch_aware: bool = False):
    """(tile, splits) for a forward/dgrad implicit GEMM.

    ``batch_aware`` (the CIFAR executor's 5x5 layers): a layer that splits K,
    or has <= 1024 output rows (batch <= 4 at 16x16), is latency-bound -- a
    few microseconds of DMA-ring fill per workgroup, whatever the work -- so it
    takes 64x64 tiles when M <= 1024 (128x64 otherwise) and doubles the splits
    while the grid is under 256 workgroups, each split keeps >= 6 K-steps of
    64 and splits <= 16.  Measured per layer at batch 4 / 32 / 128
    (scripts/sweep_small_batch.py, profiles/r6_sweep_small_batch.txt): batch 4
    dgrad3 15.9 -> 10.9 us, fwd4 16.4 -> 11.9 us; batch 32 fwd3 18.7 -> 16.5 us;
    every batch-128 plan unchanged.

    Otherwise the batch-128 rule: the biggest tile the
    channel count allows, then split-K until the grid covers the 256 CUs
    (keeping >= 8 K-steps of 64 per split).  Split-K layers run on 128x64
    tiles with half the splits (half the fp32 slab bytes written and combined,
    twice the workgroups per split: fwd4 / dgrad4 at batch 128, 0.3306 vs
    0.3347 ms/step, profiles/r3_split128x64_ab.txt), and a 128x128 layer whose
    128x64 tiles already fill the chip takes no split at all (no slab round
    trip, no combine: fwd3 28.5 -> 24.7 us)."""
    tile, splits = _fwd_plan_b128(M, N, K)
    if not batch_aware or (splits == 1 and M > 1024):
        return tile, splits
    tile = 1 if M <= 1024 else 2
    bm, bn = _FWD_TILES[tile]
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    ksteps = (K + 63) // 64
    splits = 1
    while tiles * splits < 256 and splits < 16 and ksteps // (splits * 2) >= 6:
        splits *= 2
    return tile, splits


def _fwd_plan_b128(M: int, N: int, K: int):
    tile = 0 if N % 128 == 0 else 2
    bm, bn = _FWD_TILES[tile]
    tiles = ((M + bm - 1) // bm) * ((N + bn - 1) // bn)
    ksteps = (K + 63) // 64
    splits = 1
    while tiles * splits < 256 and ksteps // (splits * 2) >= 8:
        splits *= 2
    if splits > 1 and tile == 0 and ((M + 127) // 128) * (N // 64) >= 256:
        return 2, 1
    if splits > 1 and tile == 0:
        return 2, max(1, splits // 2)
    return tile, splits


def _wgrad_plan(cout: int, K: int, M: int, reserve: int = 0):
    """(tile, splits) for the weight gradient.  128x128 tiles (tile 2: 4-stage
    DMA ring, fragment prefetch, one workgroup per CU) whenever Cout allows,
    else 64x64 (two per CU).  Every workgroup is one ~20 us "round", so the
    split count fills the resident slots exactly (not the next power of two:
    conv3 50 tiles x 5 splits = 250 workgroups, 26 k-steps each, beats 4 splits
    = 200 workgroups of 32 k-steps by 1.7 us), keeping >= 512 rows per split.
    ``reserve`` CUs are left to a concurrent RCCL collective (its workgroups do
    not fit beside these: parallel/comm.py).  (Rejected and removed in round 6:
    256x128 tiles, r3_wgrad_tile256_ab.txt; position-major steps,
    r5_wgrad_posm_ab.txt; the first layer from an LDS-resident region,
    r5_wgrad_c8r_ab.txt.)"""
    tile = 2 if cout % 128 == 0 else 1
    bm, bn = {2: (128, 128), 1: (64, 64)}[tile]
    slots = 2 * (256 - reserve) if tile == 1 else 256 - reserve
    tiles = (cout // bm) * ((K + bn - 1) // bn)
    # at most 128 splits: the reducer (a 32-lane group per weight) then keeps
    # its 4 loads per lane in flight at once -- the pair-packed layer 1 (2
    # tiles) at 256 splits: wgrad 8.6 us but its reduce 11.1 vs 8.8 us at 128
    # (profiles/r6_pair1_x4_ab.txt)
    splits = max(1, min(slots // tiles, M // 512, 128))
    return tile, splits


class CifarHIPExecutor:
    takes_loader = True  # gathers DeviceLoader batches on the device inside the step

    def __init__(self, model: CifarConvNet, flat, bucketer=None, max_batch: Optional[int] = None):
        if not isinstance(model, CifarConvNet):
            raise TypeError("CifarHIPExecutor needs a CifarConvNet")
        if flat.shadow is None:
            raise ValueError("CifarHIPExecutor needs FlatParams(shadow_bf16=True)")
        self.C = native()
        self.model, self.flat, self.bucketer = model, flat, bucketer
        self.dev = flat.data.device
        self.B = int(max_batch or 128)
        ch = model.channels
        self.nb = model.nblocks
        self.cins = [CIN_PAD] + list(ch[1:-1])      # kernel-side input channels per block
        self.cins_real = list(ch[:-1])
        self.couts = list(ch[1:])
        self.hs = [model.image >> i for i in range(self.nb)]
        self.nclass = model.num_classes
        self.feat = ch[-1] * model.final_hw * model.final_hw
        # flat views (walk order = registration order)
        self.p32 = flat.param_views()
        self.p16 = flat.shadow_views()
        self.g32 = flat.views_of(flat.grad)
        self.rm = [getattr(model, f"bn{i + 1}_rm") for i in range(self.nb)]
        self.rv = [getattr(model, f"bn{i + 1}_rv") for i in range(self.nb)]
        # every gradient element is overwritten each step by its producing kernel
        # (conv biases: exactly 0 under train-mode BN, zeroed once here) and
        # head_wgrad sets the participation slot: the engine skips the per-step
        # fill of the gradient buffer
        self.overwrites_grads = True
        # nothing in the backward reads a parameter once its gradient bucket is
        # complete (the dgrads read the step's flipped/transposed weight copies,
        # the BN/head kernels read gamma / the classifier before the block's
        # leaves are reported): the trainer may update each bucket on the comm
        # stream right after its all-reduce (engine.py bucket_updates)
        self.bucket_updates_safe = True
        for i in range(self.nb):
            self.g32[self._leaf(i, 1)].zero_()
        self.C.set_conv_stages(3, 0)
        # The dgrad convolutions run while the bucketed all-reduce is in flight
        # (the first bucket is launched after the last layer's wgrad).  With one
        # CU held by a workgroup of RCCL's footprint (19.7 KiB LDS, ~280
        # registers/wave; scripts/emulate_rccl.py, bench_conv.py --occupy 1) the
        # 256-workgroup streaming dgrad with the 3-stage ring (96 KiB LDS) slows
        # by 14 us (dgrad3/dgrad4 23 -> 37 us), with the 2-stage ring (64 KiB,
        # two workgroups fit a CU) by 1 us; the region dgrad (layer 2) by 1 us.
        # With a real all-reduce (world > 1) the dgrads use the 2-stage ring
        # (the measured overlap policy may choose otherwise: select_policy).
        comm = getattr(bucketer, "comm", None)
        overlapped = comm is not None and runs_collectives(comm)
        self.dgrad_stages = int(os.environ.get("DISTLEARN_DGRAD_STAGES", "2" if overlapped else "3"))
        # CUs held by the concurrent collective's workgroups (wgrad grids leave them free)
        self.cu_reserve = int(os.environ.get("DISTLEARN_CU_RESERVE",
                                             getattr(comm, "cu_reserve", 0) if overlapped else 0))
        # the last block's BN/ReLU/pool runs inside the head kernel (2048 pooled
        # features, 10 classes: the reference net), which also computes the
        # classifier's weight gradient
        self.head_pool = (self.hs[-1] // 2) ** 2 * self.couts[-1] == 2048 and self.nclass == 10
        # the FORWARD conv of an image smaller than a 128-row tile (layer 3: 8x8, two
        # images per tile) on the region kernel's whole-image tiles: 20.5 vs 24.6 us
        # (scripts/bench_conv.py), 0.2981 vs 0.3021 ms/step (profiles/r5_fwd3_region_ab.txt);
        # the dgrad of that layer stays on the streaming kernel, which hosts the side SGD
        self.fwd_region_images = True
        # the dgrad weight flip-transposes ride the head launch (blocks past the batch,
        # on the CUs its 128 blocks leave idle) instead of the step's prep launch:
        # prep 9.0 -> 4.8 us (profiles/r3_head_transposes_ab.txt)
        self.head_wgrad_fused = self.nclass == 10  # the classifier wgrad inside the BN backward reduce launch
        self.head_transposes = (self.head_pool and
                                all(self.cins[i] % 64 == 0 and self.couts[i] % 64 == 0 for i in range(1, self.nb)))
        # Reduction mode (csrc/kernels/bn_fin_dev.h).  0 = deterministic partial
        # rows + finalize kernels (bitwise run-to-run reproducible: the bitwise
        # graph-vs-eager and resume tests).  2 (default) = BN statistics and BN
        # parameter gradients accumulated with fp32 atomics striped over R = 16
        # rows (row = tile / block index mod R, zeroed by the prep kernel, summed
        # by every consumer block with all row loads in flight, overlapped with
        # its first data loads: R-fold less same-address contention than one
        # row), weight gradients on split-K slabs: 7 finalize launches fewer,
        # 0.3466 vs 0.3625 ms/step (profiles/r2_mode2_ab.txt).  Not bitwise
        # reproducible run to run (fp32 atomics); the replicas stay bitwise
        # identical (they apply the same all-reduced gradient).  (Mode 1 -- one
        # atomic row and atomic split-K weight gradients -- measured 0.495 vs
        # 0.358 ms/step, profiles/r2_mode1_timeline.txt; removed in round 6.)
        self.mode = int(os.environ.get("DISTLEARN_REDUCE_ATOMIC", "2"))
        if self.mode not in (0, 2):
            raise ValueError("DISTLEARN_REDUCE_ATOMIC must be 0 or 2")
        # a split-K dgrad's combine runs inside the BN backward reduce of the block
        # below (csrc bn_pool.hip combine_bwd_reduce): dP is produced, stored and
        # reduced by one launch (DISTLEARN_FUSE_COMBINE=0: separate kernels, the
        # reference the fused path is tested against)
        self.fuse_combine = os.environ.get("DISTLEARN_FUSE_COMBINE", "1") == "1"
        # an unsplit (region-kernel) dgrad runs the BN backward reduce of the block
        # below in its epilogue (csrc conv_fwd_bnred; DISTLEARN_DGRAD_BNRED=0: A/B)
        self.dgrad_bnred = os.environ.get("DISTLEARN_DGRAD_BNRED", "1") == "1"
        # split-K forwards combine their slices in-launch (csrc splitk_fixup): the
        # splitk_combine launch is gone (layer-4 forward 18.2 + 5.4 -> 22.6 us,
        # profiles/r6_fix_ab.txt).  DISTLEARN_FIX=2: the split-K dgrads too, their
        # reducers running the BN backward reduce of the block below -- measured
        # slower than the combine_bwd_reduce launch (dgrad4 22.9 -> 25.9, dgrad3
        # 33.5 -> 34.9 us: the reducer's chain of slice drain, counter, slice loads
        # and pool-window loads is serial latency at the kernel's tail), 0: off
        self.fix = int(os.environ.get("DISTLEARN_FIX", "1"))
        # layer 1 on pair-packed weights over a 4-channel input (csrc
        # conv_fwd_c8_kernel PAIR, make_geom_pair): forward 12.3 -> 11.1 us, step
        # 0.2946 -> 0.2929 ms (profiles/r6_pair1_ab.txt); the weight gradient in
        # the same layout (K 200 -> 120) 12.2 -> 8.8 us, step 0.2981 -> 0.2949 ms
        # median of 10 interleaved runs against the channel-padded layer 1
        # (profiles/r6_pair1_x4_ab.txt)
        self.pair1 = True
        # the update of blocks 1 .. side block - 1 rides the first layer's weight
        # gradient launch (side_update); DISTLEARN_SIDE_WGRAD1=0: off
        self.side_wgrad1 = os.environ.get("DISTLEARN_SIDE_WGRAD1", "1") == "1"
        self.atomic = self.mode > 0             # BN statistics / gradients by atomics, no finalize kernels
        # (mode 2) the last block's BN backward reduce runs inside the head kernel and
        # the classifier weight gradient rides the BN backward apply launch
        # (DISTLEARN_HEAD_REDUCE=0: bwd_reduce_head's separate launch, the tests' reference)
        self.head_reduce = (os.environ.get("DISTLEARN_HEAD_REDUCE", "1") == "1" and self.mode == 2 and self.head_pool
                            and self.couts[-1] == 512)
        self.rows = {0: 0, 2: 16}[self.mode]
        self._alloc(self.B)
        self._deferred = ()  # blocks whose weight-gradient slab reduce the update performs (defer_slab_reduce)
        # multi-node step (fuse_slab_reduces): blocks whose slabs are summed by
        # extra workgroups of their own dgrad launch, and blocks summed together
        # by one reduce-only launch after the last weight gradient
        self._ride: dict = {}
        self._merged: tuple = ()
        self._prefetched = False  # the coming step was prepared by the last update launch (arm_next_prep)
        self.prepared_ahead = 0   # steps armed that way (counted at capture)
        self._side = None    # side SGD carried by a dgrad launch (side_update)

    # ------------------------------------------------------------------ buffers
    def _alloc(self, B: int):
        d, C = self.dev, self.C
        e = lambda *s, dt=BF16: torch.empty(*s, dtype=dt, device=d)  # noqa: E731
        H0 = self.hs[0]
        # convolution inputs live in zero-bordered buffers [B, H+4, W+4, C]: the
        # producers write the interior, the kernels never bounds-test a tap
        P2 = 2 * SPAD
        # layer 1 on pair-packed weights reads a 4-channel input (8-byte pixels; the
        # wgrad's B chunk = two adjacent pixels), else the 8-channel one
        self.kin0 = 4 if self.pair1 else CIN_PAD
        self.k1 = KSIZE * ((KSIZE + 1) // 2) * 8 if self.pair1 else KSIZE * KSIZE * CIN_PAD  # layer-1 K
        self.x8 = torch.zeros(B, H0 + P2, H0 + P2, self.kin0, dtype=BF16, device=d)
        # layer-1 weights for its forward: pair-packed (two adjacent taps' 3 channels
        # per 16-byte chunk, csrc dl_common.h pack1_index with cp = -KSIZE: 120
        # instead of 200 K values per output channel, conv_fwd_c8_kernel PAIR);
        # the packers (prep, the update's tail) never write the zero pads
        self.w1_cp = -KSIZE if self.pair1 else CIN_PAD
        self.w1p = torch.zeros(self.couts[0], KSIZE * ((KSIZE + 1) // 2) * 8 if self.pair1
                               else KSIZE * KSIZE * CIN_PAD, dtype=BF16, device=d)
        self.wt = [None] + [e(self.cins[i], KSIZE, KSIZE, self.couts[i]) for i in range(1, self.nb)]
        self.y = [e(B, h, h, c) for h, c in zip(self.hs, self.couts)]
        self.p = [torch.zeros(B, h // 2 + P2, h // 2 + P2, c, dtype=BF16, device=d) if i + 1 < self.nb
                  else e(B, h // 2, h // 2, c) for i, (h, c) in enumerate(zip(self.hs, self.couts))]
        self.dP = [e(B, h // 2, h // 2, c) for h, c in zip(self.hs, self.couts)]
        # one dy buffer per block: block i's wgrad (side stream) still reads dy_i
        # while the main stream writes dy_{i-1}
        self.dYs = [torch.zeros(B, h + P2, h + P2, c, dtype=BF16, device=d) for h, c in zip(self.hs, self.couts)]
        self.coef = [torch.empty(4, c, device=d) for c in self.couts]
        self.acoef = [torch.empty(3, c, device=d) for c in self.couts]
        self.fwd_plan, self.stats = [], []
        # mode 2: R zeroed [2][C] (sum, sumsq) rows per layer in one arena, and R
        # [2][C] (dgamma, dbeta) rows per layer for the backward reduce
        R = self.rows
        per = sum(2 * R * c for c in self.couts)
        arena = torch.zeros(2 * per, device=d) if self.atomic else None
        arena_off = 0
        self.bwd_rows = [None] * self.nb
        self.dgrad_plan = [None] * self.nb
        self.bwd_blocks, self.bwd_part = [], []
        self.wplan, slab_elems, wslab_elems = [], 0, 0
        self.wslab_l = []
        for i in range(self.nb):
            h, cin, cout = self.hs[i], self.cins[i], self.couts[i]
            M = B * h * h
            K = KSIZE * KSIZE * cin
            Kw = self.k1 if i == 0 else K  # the weight gradient's K (layer 1: its packed layout)
            tile, splits = _fwd_plan(M, cout, K, batch_aware=True)
            if tile == 2 and splits == 2 and self._fix_ok(B, h, cin, cout, 2, 4):
                # combined in-launch, a 2-split forward takes 4 (two rounds of the
                # 128x64 grid; the reducer's 3 extra slice loads are all in flight):
                # batch-128 layer-4 forward 22.7 -> 20.9 us, step 0.2946 -> 0.2935 ms
                # median of 10 interleaved runs (profiles/r6_fwd4_splits_ab.txt)
                splits = 4
            self.fwd_plan.append((tile, splits))
            if splits > 1:
                slab_elems = max(slab_elems, splits * M * cout)
            if self.atomic:
                self.stats.append(arena[arena_off:arena_off + 2 * R * cout].view(R, 2, cout))
                self.bwd_rows[i] = arena[per + arena_off:per + arena_off + 2 * R * cout].view(R, 2, cout)
                arena_off += 2 * R * cout
            else:
                rows = C.conv_fwd_stat_rows(B, h, h, cin, cout, KSIZE, tile, splits)
                if splits > 1:
                    rows = max(rows, 400)  # the split-K combine launches <= ~384 blocks for any batch
                self.stats.append(torch.empty(rows, 2, cout, device=d))
            g = C.bn_bwd_blocks(B, h, h, cout)
            self.bwd_blocks.append(g)
            # (mode 0) partial rows of the BN backward reduce -- or of the fused
            # split-K combine + reduce, which writes one row per combine block
            # ... or of the next block's dgrad with the reduce in its epilogue (one row per M tile)
            gp = max(g, C.combine_bwd_reduce_blocks(B, h, h, cout), (B * (h // 2) * (h // 2) + 127) // 128) \
                if i + 1 < self.nb else g
            self.bwd_part.append(None if self.atomic else torch.empty(gp, 2, cout, device=d))
            tile_w, splits_w = _wgrad_plan(cout, Kw, M, self.cu_reserve)
            direct = splits_w == 1 and cin == self.cins_real[i]
            self.wplan.append((tile_w, splits_w, direct))
            if not direct:
                wslab_elems = max(wslab_elems, splits_w * cout * Kw)
            self.wslab_l.append(None if direct else torch.empty(splits_w * cout * Kw, device=d))
            if i > 0:
                dt, ds = _fwd_plan(M, cin, KSIZE * KSIZE * cout, batch_aware=True)
                self.dgrad_plan[i] = (dt, ds)
                if ds > 1:
                    slab_elems = max(slab_elems, ds * M * cin)
        self.slabs = torch.empty(max(slab_elems, 1), device=d)    # fwd / dgrad split-K (main stream)
        # what the step's prep kernel zeroes in mode 2: the statistics arena and the backward rows
        self.zero_ranges = []
        if self.atomic:
            self.zero_ranges.append((arena.data_ptr(), arena.numel()))
            self._arena = arena
        self.logits = torch.empty(B, self.nclass, device=d)
        self.dlogits = torch.empty(B, self.nclass, device=d)
        self.loss_b = torch.empty(B, device=d)
        self.loss = torch.zeros(1, device=d)
        self.cap = B

    # ------------------------------------------------------------------ helpers
    def _leaf(self, blk: int, j: int) -> int:
        return 4 * blk + j  # conv_w, conv_b, bn_w, bn_b

    def _transpose_args(self, with_transposes: bool):
        if not with_transposes:
            return [], [], [], []
        idx = list(range(1, self.nb))
        return ([self.p16[self._leaf(i, 0)].data_ptr() for i in idx], [self.wt[i].data_ptr() for i in idx],
                [self.couts[i] for i in idx], [self.cins[i] for i in idx])

    def _zero_args(self, train: bool):
        if not (train and self.atomic):
            return [], []
        return [p for p, _ in self.zero_ranges], [n for _, n in self.zero_ranges]

    def _prep(self, x, s: int, with_transposes: bool = False, train: bool = True) -> int:
        """ONE launch: the step's input into the zero-bordered, channel-padded
        layer-1 buffer (from a bf16 NHWC tensor, or gathered + normalised on
        the device from a :class:`~torch_distlearn_amd.data.DeviceLoader`),
        the layer-1 weight pack and (optionally) the dgrad weight transposes."""
        h = self.hs[0]
        tw = self._transpose_args(with_transposes)
        if hasattr(x, "gather_args"):  # DeviceLoader: batch selected by the device-side step counter
            B = x.batch
            if B > self.cap:
                raise ValueError(f"batch {B} > executor capacity {self.cap}")
            img, order, lab_all, lab_out, ctr, n_order, C, mean, std = x.gather_args()
            if (x.H, x.W, C) != (h, h, self.cins_real[0]):
                raise ValueError("DeviceLoader images do not match the model input")
            self.C.prep_step_gather(img, order, lab_all, lab_out, ctr, n_order, B, C, mean, std, self.x8.data_ptr(),
                                    self.kin0, h, h, SPAD, self.p32[0].data_ptr(), self.w1p.data_ptr(), self.couts[0],
                                    KSIZE * KSIZE, self.cins_real[0], self.w1_cp, *tw, *self._zero_args(train), s)
            return B
        B = x.shape[0]
        if B > self.cap:
            raise ValueError(f"batch {B} > executor capacity {self.cap}")
        if x.dim() != 4 or x.shape[-1] != self.cins_real[0] or x.dtype != BF16 or not x.is_contiguous():
            raise ValueError("CifarHIPExecutor expects contiguous NHWC bf16 input [B, H, W, 3]")
        self.C.prep_step(x.data_ptr(), self.x8.data_ptr(), B * h * h, self.cins_real[0], self.kin0, h, h, SPAD,
                         self.p32[0].data_ptr(), self.w1p.data_ptr(), self.couts[0], KSIZE * KSIZE,
                         self.cins_real[0], self.w1_cp, *tw, *self._zero_args(train), s)
        return B

    def _forward(self, B: int, s: int, train: bool, pool_last: bool = True):
        """Conv -> BN finalize -> BN/ReLU/pool per block.  ``pool_last=False``
        leaves the last block's pool to the head kernel (head_fwd_bwd_pool).
        (Block i-1's BN/ReLU/pool applied on load by block i's conv measured a
        wash -- 25.9 us for the fused conv vs 18.1 + 8.2 us, both bound by the
        one read of the pre-BN output, profiles/r4_pool_on_load_ab.txt --
        and was removed in round 6.)"""
        C = self.C
        inp = self.x8
        for i in range(self.nb):
            h, cin, cout = self.hs[i], self.cins[i], self.couts[i]
            M = B * h * h
            w = self.w1p if i == 0 else self.p16[self._leaf(i, 0)]
            t, sp = self.fwd_plan[i]
            if i == 0 and self.pair1:
                t |= 1 << 24  # pair-packed weights (csrc FwdCfg bit 24)
            img = self.fwd_region_images and h * h < 128 and 128 % (h * h) == 0
            if img:
                C.set_conv_region(2)
            try:
                if self._fix_ok(B, h, cin, cout, t, sp):
                    ntm = C.conv_fwd_fix(inp.data_ptr(), w.data_ptr(), self.y[i].data_ptr(),
                                         self.stats[i].data_ptr() if train else 0, self.slabs.data_ptr(), B, h, h,
                                         cin, cout, KSIZE, t, sp, 0, 0, 0, s)
                else:
                    ntm = C.conv_fwd(inp.data_ptr(), w.data_ptr(), self.y[i].data_ptr(),
                                     self.stats[i].data_ptr() if train else 0, self.slabs.data_ptr(), B, h, h,
                                     self.kin0 if i == 0 else cin, cout, KSIZE, t, sp, s)
            finally:
                if img:
                    C.set_conv_region(1)
            fused = train and self.atomic  # coefficients derived by the consumer kernel
            if not fused:
                C.bn_finalize(self.stats[i].data_ptr(), ntm, cout, M, self.p32[self._leaf(i, 2)].data_ptr(),
                              self.p32[self._leaf(i, 3)].data_ptr(), self.p32[self._leaf(i, 1)].data_ptr(),
                              self.rm[i].data_ptr(), self.rv[i].data_ptr(), BN_EPS, BN_MOMENTUM, 0 if train else 1,
                              self.coef[i].data_ptr(), s)
            if pool_last or i + 1 < self.nb:
                opad = SPAD if i + 1 < self.nb else 0
                if fused:
                    C.bn_relu_pool_fwd_fin(self.y[i].data_ptr(), *self._fin_args(i, M), self.p[i].data_ptr(), B, h,
                                           h, cout, opad, s)
                else:
                    C.bn_relu_pool_fwd(self.y[i].data_ptr(), self.coef[i].data_ptr(), self.p[i].data_ptr(), B, h, h,
                                       cout, opad, s)
            inp = self.p[i]

    def _fix_ok(self, B: int, h: int, cin: int, cout: int, tile: int, splits: int) -> bool:
        """Whether a split-K conv of this plan combines its slices inside the
        launch (csrc conv_fwd_fix: the tile's last-arriving slice sums them and
        runs the epilogue) instead of a combine launch.  DISTLEARN_FIX=0: off."""
        return (self.fix > 0 and splits > 1 and self.C.conv_fix_ok(B, h, h, cin, cout, KSIZE, tile, splits) == 1)

    def _slab_cp(self, i: int) -> int:
        """The weight-gradient slab layout of block i for the reducers (csrc
        slab_reduce_each Cp): the padded channel count, or -KSIZE for the
        pair-packed first layer (dl_common.h pack1_index)."""
        return self.w1_cp if i == 0 else self.cins[i]

    def _fin_args(self, i: int, M: int):
        """(sums, M, gamma, beta, conv bias, running mean, running var, eps,
        momentum, coef) of block i for the kernels that finalize the BN
        statistics themselves (mode 2)."""
        return (self.stats[i].data_ptr(), M, self.p32[self._leaf(i, 2)].data_ptr(),
                self.p32[self._leaf(i, 3)].data_ptr(), self.p32[self._leaf(i, 1)].data_ptr(), self.rm[i].data_ptr(),
                self.rv[i].data_ptr(), BN_EPS, BN_MOMENTUM, self.coef[i].data_ptr())

    # ------------------------------------------------------------------ API
    def forward_backward(self, x, labels: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One forward + backward on this node's batch (``x`` NHWC bf16 with
        int64 ``labels``, or a DeviceLoader); fp32 grads land in the flat
        gradient buffer.  Returns the mean loss (device tensor)."""
        C = self.C
        self._set_mode()
        s = torch.cuda.current_stream().cuda_stream
        ctr = 0
        if hasattr(x, "gather_args"):
            labels = x.labels_out
            ctr = x.ctr.data_ptr()  # advanced by head_wgrad after the gather read it
        if labels.dtype != torch.int64:
            raise ValueError("labels must be int64")
        if self._prefetched:  # the previous step's update launch prepared this one (arm_next_prep)
            self._prefetched = False
            if self.C.sgd_next_prep_armed():
                self.C.disarm_sgd_next_prep()
                raise RuntimeError("arm_next_prep: no update launch consumed the next-step preparation")
            if not hasattr(x, "gather_args"):
                raise RuntimeError("arm_next_prep: the prepared step must run on the same DeviceLoader")
            B = x.batch
        else:
            if self.C.sgd_next_prep_armed():  # stale (an update that raised after arm_next_prep): drop it
                self.C.disarm_sgd_next_prep()
            B = self._prep(x, s, with_transposes=not self.head_transposes)
        self._last_b = B
        self._forward(B, s, train=True, pool_last=not self.head_pool)
        nfc = 4 * self.nb
        if self.head_pool:  # the last block's BN/ReLU/pool runs inside the head kernel (writes p[-1])
            hl = self.hs[-1]
            last = self.nb - 1
            if self.atomic:
                sums, Ml, gam, bet, cb, rm, rv, eps, mom, _ = self._fin_args(last, B * hl * hl)
                fin = (sums, Ml, gam, bet, cb, rm, rv, eps, mom)
            else:
                fin = (0, 0, 0, 0, 0, 0, 0, 0.0, 0.0)
            C.head_fwd_bwd_pool_wt(self.y[-1].data_ptr(), self.coef[-1].data_ptr(), hl, hl, self.couts[-1],
                                   self.p[-1].data_ptr(), self.p32[nfc].data_ptr(), self.p32[nfc + 1].data_ptr(),
                                   labels.data_ptr(), B, self.nclass, self.logits.data_ptr(), self.dlogits.data_ptr(),
                                   self.loss_b.data_ptr(), self.dP[-1].data_ptr(), *fin,
                                   self.bwd_rows[last].data_ptr() if self.head_reduce else 0, s,
                                   *self._transpose_args(self.head_transposes), KSIZE * KSIZE)
        else:
            C.head_fwd_bwd(self.p[-1].data_ptr(), self.p32[nfc].data_ptr(), self.p32[nfc + 1].data_ptr(),
                           labels.data_ptr(), self.feat, B, self.nclass, self.logits.data_ptr(),
                           self.dlogits.data_ptr(), self.loss_b.data_ptr(), self.dP[-1].data_ptr(), s)
        head_args = (self.p[-1].data_ptr(), self.dlogits.data_ptr(), self.loss_b.data_ptr(), self.feat,
                     self.nclass, self.g32[nfc].data_ptr(), self.g32[nfc + 1].data_ptr(), self.loss.data_ptr(),
                     self.flat.slot.data_ptr(), ctr)
        if not self.head_wgrad_fused:
            h_, dl_, lb_, F_, nc_, dw_, db_, loss_, slot_, ctr_ = head_args
            C.head_wgrad(h_, dl_, lb_, F_, B, nc_, dw_, db_, loss_, slot_, ctr_, s)
            self._ready(nfc)
            self._ready(nfc + 1)
        dp_splits = 0   # > 0: dP[i] is still in the split-K slabs of block i+1's dgrad (fused combine)
        dp_reduced = 0  # > 0: block i+1's dgrad epilogue already reduced dP[i] (rows written)
        for i in reversed(range(self.nb)):
            T = self.bwd_blocks[i]  # partial rows written by this block's backward reduce
            h, cin, cout = self.hs[i], self.cins[i], self.couts[i]
            M = B * h * h
            G = self.bwd_blocks[i]
            dY = self.dYs[i]
            # mode 0: deterministic partial rows; mode 2: R striped rows (the apply
            # kernel writes the totals to the flat gradient)
            part = self.bwd_rows[i] if self.atomic else self.bwd_part[i]
            if i == self.nb - 1 and self.head_reduce:
                pass  # reduced inside the head kernel; the classifier wgrad rides the apply launch
            elif dp_reduced:
                T = dp_reduced  # reduced in block i+1's dgrad epilogue
                dp_reduced = 0
            elif i == self.nb - 1 and self.head_wgrad_fused:
                # one launch: this block's BN backward reduce + the classifier weight gradient
                C.bn_bwd_reduce_head(self.y[i].data_ptr(), self.dP[i].data_ptr(), self.coef[i].data_ptr(),
                                     part.data_ptr(), B, h, h, cout, G, *head_args, s)
                self._ready(nfc)
                self._ready(nfc + 1)
            elif dp_splits:
                # one launch: block i+1's dgrad split-K combine (dP[i]) + this block's BN backward reduce
                T = C.combine_bwd_reduce(self.slabs.data_ptr(), dp_splits, self.dP[i].data_ptr(),
                                         self.y[i].data_ptr(), self.coef[i].data_ptr(), part.data_ptr(), B, h, h, cout,
                                         s)
                dp_splits = 0
            else:
                C.bn_relu_pool_bwd_reduce(self.y[i].data_ptr(), self.dP[i].data_ptr(), self.coef[i].data_ptr(),
                                          part.data_ptr(), B, h, h, cout, G, s)
            if self.atomic:
                dgo, dbo = self.g32[self._leaf(i, 2)].data_ptr(), self.g32[self._leaf(i, 3)].data_ptr()
                if i == self.nb - 1 and self.head_reduce:
                    h_, dl_, lb_, F_, nc_, dw_, db_, loss_, slot_, ctr_ = head_args
                    C.bn_bwd_apply_head(self.y[i].data_ptr(), self.dP[i].data_ptr(), self.coef[i].data_ptr(),
                                        part.data_ptr(), self.p32[self._leaf(i, 2)].data_ptr(), M, dY.data_ptr(), B, h,
                                        h, cout, SPAD, dgo, dbo, h_, dl_, lb_, F_, nc_, dw_, db_, loss_, slot_, ctr_, s)
                    self._ready(nfc)
                    self._ready(nfc + 1)
                else:
                    C.bn_relu_pool_bwd_apply_sums(self.y[i].data_ptr(), self.dP[i].data_ptr(),
                                                  self.coef[i].data_ptr(), part.data_ptr(),
                                                  self.p32[self._leaf(i, 2)].data_ptr(), M, dY.data_ptr(), B, h, h,
                                                  cout, SPAD, dgo, dbo, s)
            else:
                C.bn_bwd_finalize(self.bwd_part[i].data_ptr(), T, cout, M, self.p32[self._leaf(i, 2)].data_ptr(),
                                  self.coef[i].data_ptr(), self.g32[self._leaf(i, 2)].data_ptr(),
                                  self.g32[self._leaf(i, 3)].data_ptr(), self.acoef[i].data_ptr(), s)
                C.bn_relu_pool_bwd_apply(self.y[i].data_ptr(), self.dP[i].data_ptr(), self.coef[i].data_ptr(),
                                         self.acoef[i].data_ptr(), dY.data_ptr(), B, h, h, cout, SPAD, s)
            xin = self.x8 if i == 0 else self.p[i - 1]
            K = self.k1 if i == 0 else KSIZE * KSIZE * cin
            kcin = self.kin0 if i == 0 else cin
            tile, splits, direct = self.wplan[i]
            wtile = tile | (1 << 24) if i == 0 and self.pair1 else tile  # pair-packed layer 1 (csrc make_geom_pair)
            gw = self.g32[self._leaf(i, 0)]
            if i == 0 and self._side is not None and self._side["w"] is not None:
                self._arm_side(self._side["w"])  # this launch also updates blocks 1 .. side block - 1
            if direct:
                C.conv_wgrad(dY.data_ptr(), xin.data_ptr(), gw.data_ptr(), B, h, h, kcin, cout, KSIZE, 1, K, wtile, 0, s)
            else:
                slab = self.wslab_l[i]
                C.conv_wgrad(dY.data_ptr(), xin.data_ptr(), slab.data_ptr(), B, h, h, kcin, cout, KSIZE, splits, K,
                             wtile, 0, s)
                if i in self._deferred:
                    pass  # summed by the update kernel (defer_slab_reduce)
                elif i in self._ride:
                    pass  # summed by extra workgroups of this block's dgrad (fuse_slab_reduces)
                elif i in self._merged:
                    if i == self._merged[0]:  # the last merged block's wgrad: one launch sums them all
                        self._reduce_merged(s)
                else:
                    C.slab_reduce(slab.data_ptr(), gw.data_ptr(), splits, cout, KSIZE * KSIZE, self._slab_cp(i),
                                  self.cins_real[i], s)
            # conv bias grad: exactly 0 under train-mode BN (zeroed once at construction)
            if i in self._ride or (i in self._merged and i != self._merged[0]):
                pass  # ready once the launch that sums its slabs is enqueued
            else:
                for b in (self._merged if i in self._merged else (i,)):
                    for j in range(4):
                        self._ready(self._leaf(b, j))
            if i > 0:
                dt, ds = self.dgrad_plan[i]
                if self.dgrad_stages != 3:
                    C.set_conv_stages(self.dgrad_stages, 0)
                fix = self.fix >= 2 and self._fix_ok(B, h, cout, cin, dt, ds)
                keep = self.fuse_combine and ds in (2, 4, 8, 16) and not fix
                bnred = self.dgrad_bnred and ds == 1 and not keep and self._region_dgrad(i, B)
                prt = self.bwd_rows[i - 1] if self.atomic else self.bwd_part[i - 1]
                if bnred:
                    dp_reduced = C.conv_fwd_bnred(dY.data_ptr(), self.wt[i].data_ptr(), self.dP[i - 1].data_ptr(), B,
                                                  h, h, cout, cin, KSIZE, dt, self.y[i - 1].data_ptr(),
                                                  self.coef[i - 1].data_ptr(), prt.data_ptr(), s)
                else:
                    if self._side is not None and i == self._side["block"]:
                        self._arm_side()  # this launch also runs the update of blocks >= i
                    elif i in self._ride:
                        C.set_conv_side_reduce(*self._ride[i])  # ... or sums this block's weight-gradient slabs
                    if fix:
                        # split-K slices combined inside the launch, whose reducers also
                        # run block i-1's BN backward reduce (no combine_bwd_reduce launch)
                        dp_reduced = C.conv_fwd_fix(dY.data_ptr(), self.wt[i].data_ptr(), self.dP[i - 1].data_ptr(),
                                                    0, self.slabs.data_ptr(), B, h, h, cout, cin, KSIZE, dt, ds,
                                                    self.y[i - 1].data_ptr(), self.coef[i - 1].data_ptr(),
                                                    prt.data_ptr(), s)
                    else:
                        C.conv_fwd(dY.data_ptr(), self.wt[i].data_ptr(), self.dP[i - 1].data_ptr(), 0,
                                   self.slabs.data_ptr(), B, h, h, cout, cin, KSIZE, dt | ((1 << 20) if keep else 0),
                                   ds, s)
                    if i in self._ride:
                        for j in range(4):
                            self._ready(self._leaf(i, j))
                dp_splits = ds if keep else 0
                if self.dgrad_stages != 3:
                    C.set_conv_stages(3, 0)
        return self.loss[0]

    def policies(self) -> dict:
        """Candidate overlap policies for DataParallelTrainer.select_policy
        (world > 1): "full" = full-chip grids and 3-stage dgrads (fastest when
        nothing else holds a CU), "reserve" = 2-stage dgrads and wgrad grids
        that leave the RCCL channel cap of CUs free (what the single-CU
        emulation favoured), "wreserve" = those wgrad grids with 3-stage
        dgrads.  Empty when DISTLEARN_DGRAD_STAGES /
        DISTLEARN_CU_RESERVE pin the policy."""
        if "DISTLEARN_DGRAD_STAGES" in os.environ or "DISTLEARN_CU_RESERVE" in os.environ:
            return {}
        from ..parallel.comm import rccl_channel_cap

        comm = getattr(self.bucketer, "comm", None)
        cap = getattr(comm, "cu_reserve", 0) or rccl_channel_cap()
        # "wreserve": the wgrad grids leave the cap free, the dgrads keep 3 stages -- with
        # 32 CUs held on one GPU 0.3297-0.3300 ms/step vs full 0.3543-0.3619 and reserve
        # 0.3362-0.3380 (profiles/r6_nworld_policy_hold.txt)
        return {"full": {"dgrad_stages": 3, "cu_reserve": 0}, "reserve": {"dgrad_stages": 2, "cu_reserve": int(cap)},
                "wreserve": {"dgrad_stages": 3, "cu_reserve": int(cap)}}

    def set_policy(self, dgrad_stages: int, cu_reserve: int) -> None:
        """Switch the overlap policy (re-plans the weight-gradient grids and
        re-allocates the workspaces: graphs captured before are invalid, and
        a trainer that deferred the slab reduces calls defer_slab_reduce
        again for the new slabs)."""
        self.dgrad_stages, self.cu_reserve = int(dgrad_stages), int(cu_reserve)
        self._alloc(self.B)
        self._deferred = ()
        self._side = None
        self._ride, self._merged = {}, ()

    def side_update(self, lr_fn, momentum: float, weight_decay: float, mom, slot, block: Optional[int] = None):
        """Run the SGD update of every parameter from block ``block``'s conv
        weight to the end of the flat buffer (blocks >= block, the
        classifier) inside that block's dgrad launch, as extra workgroups on
        the CUs its one-workgroup-per-CU grid leaves free (csrc
        set_conv_side_sgd): their gradients are final by then (weight
        gradients in the flat buffer or, deferred, in their slabs) and nothing
        later in the step reads them.  One node only (after
        :meth:`defer_slab_reduce`).  Returns the flat element range [lo, hi)
        the final update must skip, or None when the block's dgrad is not a
        streaming launch."""
        nb = self.nb
        if block is None:
            block = nb - 2
        if not (0 < block < nb) or self.flat.shadow is None:
            return None
        if not self._dgrad_hosts_side_job(block):
            return None
        f = self.flat
        lo, hi = f.offsets[self._leaf(block, 0)], f.total
        base = f.data.data_ptr()
        slabs = [(f.offsets[self._leaf(i, 0)], f.numels[self._leaf(i, 0)], self.wslab_l[i].data_ptr(),
                  self.wplan[i][1]) for i in self._deferred if i >= block]
        if any(self.cins[i] != self.cins_real[i] for i in self._deferred if i >= block):
            return None
        slabs.sort()
        args = (base, f.grad.data_ptr(), 0 if mom is None else mom.data_ptr(), f.shadow.data_ptr(),
                0 if slot is None else slot.data_ptr())
        pack = lambda sl: ([o for o, _, _, _ in sl], [n for _, n, _, _ in sl],  # noqa: E731
                           [t for _, _, t, _ in sl], [k for _, _, _, k in sl])
        self._side = {"block": block, "lr": lr_fn, "args": args, "mw": (float(momentum), float(weight_decay)),
                      "range": (lo, hi), "slabs": pack(slabs), "w": None}
        # ... and the blocks before it down to block 1 ride the first layer's
        # weight-gradient launch (the last launch before the update: every one of
        # their gradients is final by then, csrc conv_wgrad_g side job), so the
        # final update is left with block 0 and its slab tail
        # (profiles/r6_side_wgrad1_ab.txt)
        lo1 = f.offsets[self._leaf(1, 0)]
        sl1 = [(f.offsets[self._leaf(i, 0)], f.numels[self._leaf(i, 0)], self.wslab_l[i].data_ptr(),
                self.wplan[i][1]) for i in self._deferred if 1 <= i < block]
        if block > 1 and self.side_wgrad1 and all(self.cins[i] == self.cins_real[i] for i in self._deferred
                                                  if 1 <= i < block):
            self._side["w"] = {"range": (lo1, lo), "slabs": pack(sorted(sl1))}
            return lo1, hi
        return lo, hi

    def _dgrad_hosts_side_job(self, block: int) -> bool:
        """Whether block ``block``'s dgrad is a streaming conv launch that can
        carry extra workgroups (csrc SgdJob side job): not the region kernel
        (its dynamic LDS leaves no room beside it) and not the region dgrad
        with the fused BN reduce."""
        if not 0 < block < self.nb:
            return False
        dt, ds = self.dgrad_plan[block]
        h, cout, cin = self.hs[block], self.couts[block], self.cins[block]
        if self.C.conv_region_ok(self.B, h, h, cout, cin, KSIZE, dt, ds):
            return False
        keep = self.fuse_combine and ds in (2, 4, 8, 16)
        return not (self.dgrad_bnred and ds == 1 and not keep)

    def fuse_slab_reduces(self) -> dict:
        """Multi-node step: the weight gradients are all-reduced, so their
        split-K slabs must be summed before the bucket holding them launches
        (the one-node update sums them itself instead: defer_slab_reduce).
        Rather than one slab_reduce launch per layer, a layer whose dgrad is a
        streaming launch has its slabs summed by extra workgroups of that
        dgrad (csrc set_conv_side_reduce, on the CUs its grid leaves free),
        and the other layers are summed together by ONE reduce-only launch
        after the last of their weight gradients (slab_reduce_multi: up to 4
        unpadded ranges + the first layer's channel-padded 128-way slabs).
        Every sum is bitwise the stand-alone reduce's (sgd_dev.h).  A layer's
        gradients are reported to the bucketer once the launch that sums them
        is enqueued (CIFAR: blocks 1-2 share the last bucket, so merging them
        delays no all-reduce).  Returns {"ride": [...], "merged": [...]}."""
        self._ride, self._merged = {}, ()
        f = self.flat
        slab_blocks = [i for i in range(self.nb) if not self.wplan[i][2]]
        unpadded = lambda i: self.cins[i] == self.cins_real[i] and self.wplan[i][1] < 32  # noqa: E731
        ride = [i for i in slab_blocks if unpadded(i) and self._dgrad_hosts_side_job(i)]
        rest = [i for i in slab_blocks if i not in ride]
        inplace = [i for i in rest if unpadded(i)][:4]
        padded = [i for i in rest if not unpadded(i)][:1]
        for i in ride:
            lf = self._leaf(i, 0)
            off, n = f.offsets[lf], f.numels[lf]
            self._ride[i] = (f.grad.data_ptr(), off, off + n, [off], [n], [self.wslab_l[i].data_ptr()],
                             [self.wplan[i][1]], 0)
        merged = sorted(inplace + padded)
        if merged:
            lfs = {i: self._leaf(i, 0) for i in merged}
            tail, tslab = [], 0
            if padded:
                i = padded[0]
                tail = [f.offsets[lfs[i]], f.numels[lfs[i]], self.wplan[i][1], self.couts[i], KSIZE * KSIZE,
                        self._slab_cp(i), self.cins_real[i]]
                tslab = self.wslab_l[i].data_ptr()
            self._merged_args = (f.grad.data_ptr(), f.total, [f.offsets[lfs[i]] for i in inplace],
                                 [f.numels[lfs[i]] for i in inplace], [self.wslab_l[i].data_ptr() for i in inplace],
                                 [self.wplan[i][1] for i in inplace], tail, tslab)
            self._merged = tuple(merged)  # ascending: [0] is the last one the backward reaches
        return {"ride": sorted(self._ride), "merged": list(self._merged)}

    def _reduce_merged(self, s: int) -> None:
        self.C.slab_reduce_multi(*self._merged_args, s)

    def _arm_side(self, job: Optional[dict] = None) -> None:
        sd = self._side
        job = job or sd
        p, g, mom, p16, slot = sd["args"]
        mo, wd = sd["mw"]
        lo, hi = job["range"]
        self.C.set_conv_side_sgd(p, g, mom, p16, slot, float(sd["lr"]()), mo, wd, lo, hi, *job["slabs"],
                                 0)  # 0: one float4 per thread over the range

    def defer_slab_reduce(self):
        """Leave every split-K weight gradient in its slabs: the slab_reduce
        launches are skipped and the fused SGD sums the slabs itself -- in
        place where the slab layout is the weight's (no channel padding, < 32
        splits), and the first layer's channel-padded 128-way slabs in extra
        blocks of the same launch (flat.py flat_sgd_ ``slabs``; bitwise the
        same sums).  Only for a trainer that all-reduces nothing (one node):
        the flat gradient of those weights is then never written.
        Returns [(leaf, slab, splits, Cout, taps, Cp, C)] for the update."""
        taps = KSIZE * KSIZE
        blocks = [i for i in range(self.nb) if not self.wplan[i][2]]
        padded = [i for i in blocks if not (self.cins[i] == self.cins_real[i] and self.wplan[i][1] < 32)]
        inplace = [i for i in blocks if i not in padded]
        # the update reads at most 4 in-place ranges (csrc sgd_dev.h kSlabRanges) and
        # reduces one padded tail; any further block keeps its stand-alone slab_reduce
        blocks = sorted(inplace[:4] + padded[:1])
        self._deferred = tuple(blocks)
        return [(self._leaf(i, 0), self.wslab_l[i], self.wplan[i][1], self.couts[i], taps, self._slab_cp(i),
                 self.cins_real[i]) for i in blocks]

    def arm_next_prep(self, loader) -> bool:
        """Let the coming update launch (flat_sgd_ with the deferred slabs)
        prepare the NEXT step on ``loader`` in extra workgroups: gather +
        normalise its batch into the layer-1 buffer, zero its accumulators,
        and write the updated first-layer weights straight into their packed
        operand (the update's tail range) -- so the next :meth:`forward_backward`
        skips its prep launch.  For consecutive steps of an unrolled graph
        (engine.py _capture_multi); the step counter the gather reads was
        advanced by this step's head kernel.  False (nothing armed) when the
        update cannot carry it: the first layer's slab reduce not deferred,
        the dgrad transposes in the prep launch, no device loader."""
        if (not hasattr(loader, "gather_args") or self.cins[0] == self.cins_real[0]
                or not self.head_transposes or loader.batch > self.cap):
            return False
        h = self.hs[0]
        img, order, lab_all, lab_out, ctr, n_order, C, mean, std = loader.gather_args()
        if (loader.H, loader.W, C) != (h, h, self.cins_real[0]):
            return False
        lf = self._leaf(0, 0)
        self.C.arm_sgd_next_prep(img, order, lab_all, lab_out, ctr, n_order, loader.batch, C, mean, std,
                                 self.x8.data_ptr(), self.kin0, h, h, SPAD, *self._zero_args(True),
                                 self.w1p.data_ptr(), self.w1_cp, self.flat.offsets[lf] - HEADER, self.flat.numels[lf])
        self._prefetched = True
        self.prepared_ahead += 1
        return True

    def _region_dgrad(self, i: int, B: int) -> bool:
        """Whether block i's (unsplit) dgrad runs on the region (tap-reuse)
        kernel, the one with the fused BN-reduce epilogue (asked from the
        native dispatch, csrc conv_region_ok)."""
        h, cout, cin = self.hs[i], self.couts[i], self.cins[i]
        return bool(self.C.conv_region_ok(B, h, h, cout, cin, KSIZE, self.dgrad_plan[i][0]))

    def _set_mode(self) -> None:
        """The reduction mode lives in device globals shared by every executor
        of the process: (re)select this executor's row count (a blocking symbol
        copy -- never issued while a hipGraph is being captured; a captured step
        replays with the mode that was active at capture)."""
        if self.C.reduce_atomic() != self.rows and not torch.cuda.is_current_stream_capturing():
            self.C.set_reduce_atomic(self.rows)

    def last_logits(self) -> torch.Tensor:
        return self.logits[:self._last_b]

    def _ready(self, leaf: int):
        if self.bucketer is not None:
            self.bucketer.mark_leaf_ready(leaf)

    @torch.no_grad()
    def predict(self, x: torch.Tensor, batch_stats: bool = False) -> torch.Tensor:
        """Forward only; returns log-probabilities [B, classes] (fp32).  Eval
        mode (running BN statistics) by default; ``batch_stats=True``
        normalises with the batch's own statistics, the way the reference's
        AsyncEA tester evaluates a center snapshot (its functional BN stays in
        training mode: examples/Model.lua:56-66, EASGD_tester.lua:109-159) --
        the running statistics are left as they were."""
        s = stream_handle()
        if batch_stats:
            self._set_mode()
        B = self._prep(x, s, train=batch_stats)
        if batch_stats:
            saved = [(t, t.clone()) for t in self.rm + self.rv]
        self._forward(B, s, train=batch_stats)
        if batch_stats:
            for t, v in saved:
                t.copy_(v)
        nfc = 4 * self.nb
        self.C.head_fwd_bwd(self.p[-1].data_ptr(), self.p32[nfc].data_ptr(), self.p32[nfc + 1].data_ptr(), 0,
                            self.feat, B, self.nclass, self.logits.data_ptr(), 0, 0, 0, s)
        return self.logits[:B].clone()
