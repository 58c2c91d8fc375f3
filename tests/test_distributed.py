"""CPU: the multi-GPU control flow under torch.distributed gloo, world_size 2 (and 3).

The collectives (all_gather_into_tensor of feature row bands and of the packed
(min, argmin) partials) and the ordered merge are exercised with the CPU
oracle standing in for the per-rank GPU compute; the merge rule is the one the
HIP argmin_merge kernel implements (strict `<` in shard order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from scenedepthestimation_amd.parallel import (allreduce_max_, gather_disparity_rows, gather_partials,
                                                pairs_for_rank, row_band, shard_range)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_shard_ranges_partition():
    for D in (1, 7, 64, 192, 512):
        for n in (1, 2, 3, 4, 8):
            if n > D:
                continue
            rs = [shard_range(D, n, s) for s in range(n)]
            assert rs[0][0] == 0 and rs[-1][1] == D
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert all(b > a for a, b in rs)
    for H in (1, 5, 1024, 1030):
        for n in (1, 2, 3, 8):
            bands = [row_band(H, n, s) for s in range(n)]
            covered = sum(r1 - r0 for r0, r1, _ in bands)
            assert covered == H and all(r1 - r0 <= rpb for r0, r1, rpb in bands)
    assert pairs_for_rank(18, 8, 0) == [0, 8, 16] and pairs_for_rank(18, 8, 7) == [7, 15]


def _merge_reference(mins, args):
    best, arg = mins[0].clone(), args[0].clone()
    for s in range(1, mins.shape[0]):
        take = mins[s] < best
        best[take], arg[take] = mins[s][take], args[s][take]
    return arg.to(torch.float32)


def _worker(rank, world, port, fl, fr, D, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        d0, d1 = shard_range(D, world, rank)
        mn, am = oracle.cv_wta_shard(fl, fr, d0, d1)
        mins, args = gather_partials(torch.from_numpy(mn), torch.from_numpy(am), world)
        disp = _merge_reference(mins, args).numpy()
        # feature row bands: each rank contributes its band, all ranks get the full map
        H = fl.shape[0]
        r0, r1, rpb = row_band(H, world, rank)
        band = torch.zeros((rpb,) + fl.shape[1:])
        band[: r1 - r0] = torch.from_numpy(fl[r0:r1])
        full = torch.empty((world * rpb,) + fl.shape[1:])
        dist.all_gather_into_tensor(full, band)
        ok_rows = bool(np.array_equal(full[:H].numpy(), fl))
        q.put((rank, disp, ok_rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_disparity_sharded_merge_is_bit_exact(oracle, world):
    rng = np.random.default_rng(world)
    H, W, D = 5, 70, 24
    fl = rng.standard_normal((H, W, 64)).astype(np.float32)
    fr = rng.standard_normal((H, W, 64)).astype(np.float32)
    fr[:, 30:40] = fr[:, 10:20]               # exact cost ties straddling shard boundaries
    fl /= np.linalg.norm(fl, axis=-1, keepdims=True)
    fr /= np.linalg.norm(fr, axis=-1, keepdims=True)
    ref = oracle.WTA1(oracle.compute_cost_volume(fl, fr, D))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fl, fr, D, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, disp, ok_rows in res:
        assert ok_rows, rank
        assert np.array_equal(disp, ref), rank


def _rowband_worker(rank, world, port, fl, fr, D, q):
    """RowBandMatcher's protocol with the oracle standing in for the GPU: per-layer MAX all-reduce of
    bound words (each rank starts from its band's own bound), CV+WTA over all D on the band's rows,
    one all-gather of the disparity rows."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle
        H, W = fl.shape[:2]
        r0, r1, rpb = row_band(H, world, rank)
        words = torch.zeros((2, 64))
        words[:, 0] = float(np.abs(fl[r0:r1]).max()) if r1 > r0 else 0.0
        for _ in range(4):                       # the tower's L - 1 bound stages
            allreduce_max_(words)
        band = torch.zeros((rpb, W))
        if r1 > r0:
            mn, am = oracle.cv_wta_shard(fl[r0:r1], fr[r0:r1], 0, D)
            band[: r1 - r0] = torch.from_numpy(am.astype(np.float32))
        disp = gather_disparity_rows(band, H, world).numpy()
        q.put((rank, disp, float(words[0, 0])))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,H", [(2, 7), (3, 8), (4, 3)])
def test_row_band_split_is_bit_exact(oracle, world, H):
    rng = np.random.default_rng(world * 10 + H)
    W, D = 60, 20
    fl = rng.standard_normal((H, W, 64)).astype(np.float32)
    fr = rng.standard_normal((H, W, 64)).astype(np.float32)
    fl /= np.linalg.norm(fl, axis=-1, keepdims=True)
    fr /= np.linalg.norm(fr, axis=-1, keepdims=True)
    ref = oracle.WTA1(oracle.compute_cost_volume(fl, fr, D))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rowband_worker, args=(r, world, port, fl, fr, D, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, disp, w0 in res:
        assert np.array_equal(disp, ref), rank
        assert w0 == np.float32(np.abs(fl).max())          # every rank ends with the whole image's bound
