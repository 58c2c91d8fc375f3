"""Multi-GPU execution: one process per GPU, torch.distributed over RCCL (xGMI).

The reference has no parallelism; two schemes are added:

* pair data-parallel (config 4): rank r matches pairs r, r+N, ...; no
  collective on the data path (``pairs_for_rank``).
* disparity-sharded cost volume (config 5, north star): rank r owns the
  disparity block ``shard_range(D, N, r)``.  Each rank computes the MC-CNN
  features of a band of rows (+ the tower's halo) and one
  ``all_gather_into_tensor`` assembles the full feature maps; each rank runs the
  fused cost volume + first-min over its block, and a single all-gather of the
  8-byte per-pixel partials (min f32, argmin i32) feeds an ordered merge
  (strict `<` in rank order == lowest d on ties), so the result is bit-identical
  to WTA1(compute_cost_volume(...)) on one device.

* disparity-sharded with the tower replicated (``ReplicatedDisparityShardedMatcher``): every
  rank runs the whole tower, its disparity block of the fused CV + first-min, and the ONE
  all-gather of the 8-byte partials -- no feature exchange.
* row-band split (config 5's zero-exchange alternative, ``RowBandMatcher``):
  rank r owns image rows ``row_band(H, N, r)`` and computes the tower on them
  (+ halo; bound words all-reduced, 4 B per layer) and the fused cost volume +
  WTA over ALL disparities for its rows -- a row's costs need only that row of
  both feature maps, so no feature crosses xGMI; one all-gather of the 4-byte
  disparity rows assembles the map.  Same bits as one device.

The collectives are plain torch.distributed calls, so the same code runs on
gloo (CPU tests; device tensors staged through host memory, which is how the one-GPU
multi-process tests run the real classes) and nccl (= RCCL on ROCm).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def shard_range(D: int, nshards: int, s: int):
    """Contiguous, ordered disparity block of shard s: [s*D//n, (s+1)*D//n)."""
    if not 0 <= s < nshards:
        raise ValueError("shard index out of range")
    return (s * D) // nshards, ((s + 1) * D) // nshards


def row_band(H: int, nshards: int, s: int):
    """Equal-height row bands (the last may be short, trailing ones may be empty) -> (r0, r1,
    rows_per_band).  Bands start on even rows: the Winograd tower ("f16x3w") computes 2 x 2
    output blocks aligned to its input's origin, so only an even band start gives every pixel
    the block position -- and the bits -- it has in the whole image."""
    rpb = (H + nshards - 1) // nshards
    rpb += rpb & 1
    r0 = min(H, s * rpb)
    return r0, min(H, r0 + rpb), rpb


def pairs_for_rank(npairs: int, world: int, rank: int):
    return list(range(rank, npairs, world))


def init_from_env(backend: str | None = None):
    """Initialise torch.distributed from torchrun's env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_*).

    backend: "nccl" (= RCCL on ROCm; one GPU per rank, cuda:LOCAL_RANK) or "gloo" (collectives on host
    tensors, device tensors staged through host memory; ranks may share a GPU: cuda:LOCAL_RANK mod
    the device count).  Default: the SDE_DIST_BACKEND environment variable, else nccl with a GPU and
    gloo without -- so the multi-rank paths can be exercised as fresh processes on a one-GPU box."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = os.environ.get("SDE_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend not in ("nccl", "gloo"):
        raise ValueError(f"backend must be nccl or gloo (got {backend!r})")
    if torch.cuda.is_available():
        torch.cuda.set_device(local if backend == "nccl" else local % torch.cuda.device_count())
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(backend=backend, init_method="env://", world_size=world, rank=rank)
    return rank, world, local


def _host_staged(t: torch.Tensor, group=None) -> bool:
    """gloo collectives take host tensors: device tensors are staged through host memory (the CPU
    tests and the one-GPU multi-process tests); nccl (= RCCL) takes them as they are."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_gather_into(out: torch.Tensor, inp: torch.Tensor, group=None):
    """dist.all_gather_into_tensor, host-staged on gloo."""
    if _host_staged(inp, group):
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)
    return out


def gather_partials(min_local: torch.Tensor, arg_local: torch.Tensor, world: int, group=None):
    """One all-gather of the per-pixel (min f32, argmin i32) partials -> ([N,H,W] f32, [N,H,W] i32)."""
    shape = tuple(min_local.shape)
    npix = min_local.numel()
    packed = torch.empty((2, npix), dtype=torch.int32, device=min_local.device)
    packed[0] = min_local.reshape(-1).view(torch.int32)
    packed[1] = arg_local.reshape(-1)
    out = torch.empty((world * 2, npix), dtype=torch.int32, device=min_local.device)   # concatenated form
    all_gather_into(out, packed, group)
    out = out.view(world, 2, npix)
    mins = out[:, 0].contiguous().view(torch.float32).reshape((world,) + shape)
    args = out[:, 1].contiguous().reshape((world,) + shape)
    return mins, args


def gather_row_bands(band: torch.Tensor, full: torch.Tensor, world: int, group=None):
    """All-gather equal-height row bands [rpb, ...] into full [world*rpb, ...]."""
    return all_gather_into(full, band, group)


def allreduce_max_(words: torch.Tensor, group=None):
    """In-place MAX all-reduce of the f16x3 bound words (non-negative floats)."""
    if _host_staged(words, group):
        w = words.cpu()
        dist.all_reduce(w, op=dist.ReduceOp.MAX, group=group)
        words.copy_(w)
    else:
        dist.all_reduce(words, op=dist.ReduceOp.MAX, group=group)
    return words


class DisparityShardedMatcher:
    """Config 5: features from row bands + all-gather, disparity-sharded fused CV/WTA + all-gather merge.

    The tower runs on this rank's row band of both images (band_tower); the f16x3 bound words are
    all-reduced (MAX) after the image bound and after every layer, so each rank scales every layer
    by the whole image's bound and its band's features are bit-identical to the single-device
    tower's rows."""

    def __init__(self, H, W, D, rank, world, weights=None, nlayers=5, nf=64, group=None, tower_precision="f16x3"):
        from .pipeline import StereoMatcher
        self.H, self.W, self.D = H, W, D
        self.rank, self.world, self.group = rank, world, group
        self.d_range = shard_range(D, world, rank)
        self.m = StereoMatcher(H, W, D, weights=weights, nlayers=nlayers, nf=nf, d_range=self.d_range,
                               tower_precision=tower_precision)
        self.r0, self.r1, self.rpb = row_band(H, world, rank)
        dev = self.m.device
        L = nlayers
        self.band = torch.zeros((2, self.rpb, W, nf), dtype=torch.float32, device=dev)
        hb = self.r1 - self.r0
        # the band's padded rows [r0, r1 + 2L) of both images, contiguous (one batched launch per layer)
        self.band_pad = torch.empty((2, hb + 2 * L, W + 2 * L), dtype=torch.float32, device=dev) if hb > 0 else None
        # a short last band writes a contiguous [2, hb, W, nf] buffer first
        self.band_out = self.band if hb == self.rpb else \
            (torch.empty((2, hb, W, nf), dtype=torch.float32, device=dev) if hb > 0 else None)
        # the band tower's workspace is band-sized (self.m's full-image tower workspace is never
        # allocated: StereoMatcher allocates it on first use, and only band_steps runs a tower here)
        from . import ops
        self.band_ws = torch.empty((max(ops.tower_batch_workspace_bytes(hb, W, 2, L, nf), 1),), dtype=torch.uint8,
                                   device=dev) if hb > 0 else None
        self.full = torch.empty((world * 2, self.rpb, W, nf), dtype=torch.float32, device=dev)
        self.disp = torch.empty((H, W), dtype=torch.float32, device=dev)

    def band_steps(self):
        """tower_steps over this rank's band (generator; see pipeline.tower_steps)."""
        from .pipeline import tower_steps
        m, L = self.m, self.m.nlayers
        if self.band_pad is None:
            return iter(())
        self.band_pad.copy_(m.img_pad2[:, self.r0:self.r1 + 2 * L])
        return tower_steps(self.band_pad, m.packed, L, self.band_out, self.band_ws, m.tower_precision, m.nf)

    def features(self):
        from . import ops
        m, L = self.m, self.m.nlayers
        ops.preprocess_u8_batch(m.img_u82, L, out=m.img_pad2, stats=m.stats2)
        if self.band_pad is not None:
            for _stage, words in self.band_steps():
                if m.tower_precision in ("f16x3", "f16x3w", "f16x3m32"):
                    allreduce_max_(words, self.group)
            if self.band_out is not self.band:
                self.band[:, :self.r1 - self.r0].copy_(self.band_out)
        elif m.tower_precision in ("f16x3", "f16x3w", "f16x3m32"):
            # an empty band still joins every bound all-reduce (same count as the other ranks)
            words = torch.zeros((2, 64), dtype=torch.float32, device=m.device)
            for _ in range(L - 1):
                allreduce_max_(words, self.group)
        all_gather_into(self.full, self.band, self.group)
        full = self.full.view(self.world, 2, self.rpb, self.W, m.nf)
        for i in range(2):
            m.feat[i].copy_(full[:, i].reshape(self.world * self.rpb, self.W, m.nf)[:self.H])
        m.split_valid = False    # assembled features: the certified call splits them itself
        return m.feat[0], m.feat[1]

    def match(self):
        from . import ops
        self.features()
        _, mn, am = self.m.cost_wta(want=("min", "argmin"))
        mins, args = gather_partials(mn, am, self.world, self.group)
        return ops.argmin_merge(mins, args, out=self.disp)


class ReplicatedDisparityShardedMatcher:
    """Config 5 with the tower replicated: every rank runs the whole tower (no feature exchange),
    the fused CV + first-min over its disparity block, and exactly ONE collective -- the
    all-gather of the 8-byte (min, argmin) partials before the ordered merge (north_star's
    scheme).  Per rank at 3840 x 2160, D = 512, N = 8: the full pair tower (~7 ms), a 64-disparity
    shard (~1 ms) and 66 MB of partials out, against the band tower's 3.7 GB feature all-gather
    (DESIGN.md sec. 6).  Same bits as one device."""

    def __init__(self, H, W, D, rank, world, weights=None, nlayers=5, nf=64, group=None, tower_precision="f16x3"):
        from .pipeline import StereoMatcher
        self.H, self.W, self.D = H, W, D
        self.rank, self.world, self.group = rank, world, group
        self.d_range = shard_range(D, world, rank)
        self.m = StereoMatcher(H, W, D, weights=weights, nlayers=nlayers, nf=nf, d_range=self.d_range,
                               tower_precision=tower_precision)
        self.disp = torch.empty((H, W), dtype=torch.float32, device=self.m.device)

    def load_images(self, left_u8, right_u8):
        self.m.load_images(left_u8, right_u8)

    def match(self):
        from . import ops
        self.m.features()
        _, mn, am = self.m.cost_wta(want=("min", "argmin"))
        mins, args = gather_partials(mn, am, self.world, self.group)
        return ops.argmin_merge(mins, args, out=self.disp)


def gather_disparity_rows(band: torch.Tensor, H: int, world: int, out: torch.Tensor | None = None, group=None):
    """All-gather equal-height [rpb, W] disparity row bands (the last band zero-padded) -> [H, W]."""
    rpb = band.shape[0]
    full = torch.empty((world * rpb,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
    all_gather_into(full, band.contiguous(), group)
    if out is None:
        return full[:H]
    out.copy_(full[:H])
    return out


class FullImages:
    """The whole pair's u8 images and padded z-normalised images (what StereoMatcher.load_images /
    preprocess hold), without the full-size feature, tower and cost-volume buffers a row band
    never uses."""

    def __init__(self, H, W, nlayers, tower_precision, device=None):
        from . import ops
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.tower_precision = tower_precision
        self.img_u82 = torch.empty((2, H, W), dtype=torch.uint8, device=self.device)
        self.img_pad2 = torch.empty((2, H + 2 * nlayers, W + 2 * nlayers), dtype=torch.float32, device=self.device)
        self.stats2 = torch.empty((2 * ops.preprocess_scratch_bytes(H, W),), dtype=torch.uint8, device=self.device)

    def load_images(self, left_u8, right_u8):
        import numpy as np
        for dst, src in zip(self.img_u82, (left_u8, right_u8)):
            t = src if isinstance(src, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(src, np.uint8))
            dst.copy_(t, non_blocking=False)


class RowBandMatcher:
    """Config 5 without a feature exchange: the tower and the fused CV + WTA (all D) on this rank's
    row band, then one all-gather of the disparity rows.  Per rank at 3840 x 2160, D = 512, N = 8:
    270 rows of tower + CV/WTA and 1 MB of disparity out, against 3.7 GB of features in for the
    disparity-sharded scheme."""

    def __init__(self, H, W, D, rank, world, weights=None, nlayers=5, nf=64, group=None, tower_precision="f16x3",
                 cv_mode="certified"):
        from .pipeline import StereoMatcher
        self.H, self.W, self.D = H, W, D
        self.rank, self.world, self.group = rank, world, group
        self.r0, self.r1, self.rpb = row_band(H, world, rank)
        self.hb = self.r1 - self.r0
        L = nlayers
        # the full images and their padded z-normalised copies live here (preprocess needs
        # whole-image statistics) -- nothing else at full size; the band matcher holds the band's
        # padded rows, features and workspaces
        self.full = FullImages(H, W, nlayers, tower_precision)
        self.band = StereoMatcher(max(self.hb, 1), W, D, weights=weights, nlayers=nlayers, nf=nf,
                                  tower_precision=tower_precision, cv_mode=cv_mode) if self.hb > 0 else None
        dev = self.full.device
        self.disp_band = torch.zeros((self.rpb, W), dtype=torch.float32, device=dev)
        self.disp = torch.empty((H, W), dtype=torch.float32, device=dev)
        self.nlayers = L

    def load_images(self, left_u8, right_u8):
        self.full.load_images(left_u8, right_u8)

    def features(self):
        from . import ops
        from .pipeline import tower_steps
        f, L = self.full, self.nlayers
        ops.preprocess_u8_batch(f.img_u82, L, out=f.img_pad2, stats=f.stats2)
        if self.band is not None:
            b = self.band
            b.img_pad2.copy_(f.img_pad2[:, self.r0:self.r1 + 2 * L])
            for _stage, words in tower_steps(b.img_pad2, b.packed, L, b.feat2, b.ws, b.tower_precision, b.nf):
                if b.tower_precision in ("f16x3", "f16x3w", "f16x3m32"):
                    allreduce_max_(words, self.group)
            b.split_valid = False
        elif f.tower_precision in ("f16x3", "f16x3w", "f16x3m32"):
            words = torch.zeros((2, 64), dtype=torch.float32, device=f.device)
            for _ in range(L - 1):
                allreduce_max_(words, self.group)

    def match(self):
        self.features()
        if self.band is not None:
            self.band.cost_wta()
            self.disp_band[: self.hb].copy_(self.band.disp)
        return gather_disparity_rows(self.disp_band, self.H, self.world, out=self.disp, group=self.group)
