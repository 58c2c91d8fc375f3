#!/usr/bin/env python
"""bench.py -- throughput of the stereo matching hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
                    [--workload north_star|cones|cv|c3|c4|c5|north_star_sgm|cones_sgm]
                    [--mode auto|pairdp|dshard|dshard_rep|rowband] [--no-cpu-baseline] [--dump-disp PATH]

A step = one stereo pair through the hot path with inputs resident in HBM:
u8 images -> z-norm + pad -> MC-CNN-fast tower (5 conv layers, f16x3 MFMA at fp32
accuracy) on both images -> fused certified cost volume + WTA over D disparities
(bit-identical to the exact NumPy-order path) -> float32 disparity.
Default workload: the north-star size 1024x1024, D = 192 (BASELINE.json).

N > 1 (one process per GPU under torchrun, RCCL).  The default --mode auto runs dshard (the north
star's disparity-sharded cost volume) for `value` on the tower + CV/WTA workloads and times the other
three schemes on the same pair after it (stages.multi_gpu_modes); on the SGM workloads (c3,
north_star_sgm: every SGM step needs all D) it runs pairdp:
  pairdp : every rank matches its own pair each step (config 4) -- weak scaling,
           no collective on the data path;
  dshard : one pair per step, disparity-sharded over the ranks with the feature
           row-band all-gather and the (min, argmin) all-gather (config 5, the
           north star's scheme) -- strong scaling;
  dshard_rep: the same with the tower replicated on every rank: exactly one
           collective, the (min, argmin) all-gather -- strong scaling;
  rowband: one pair per step, split by image rows: tower + CV/WTA over all D on
           each rank's rows, one all-gather of disparity rows (no feature
           exchange) -- strong scaling.

Rank 0 prints ONE JSON line.  `value` = H*W*D voxels of all pairs of all ranks /
the max-over-ranks wall time of the K timed steps (Mpixel-disparities/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from scenedepthestimation_amd import ops  # noqa: E402
from scenedepthestimation_amd.parallel import (DisparityShardedMatcher, ReplicatedDisparityShardedMatcher,  # noqa: E402
                                                RowBandMatcher, init_from_env)
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402
from scenedepthestimation_amd.synthetic import stereo_pair  # noqa: E402

WORKLOADS = {
    # name: (H, W, D, what)
    "north_star": (1024, 1024, 192, "tower+cv_wta"),
    "cones": (375, 450, 64, "tower+cv_wta"),
    "cv": (1024, 1024, 192, "cv_wta"),
    # BASELINE config 3: Middlebury-2014 full-resolution scale, D = 256, cross-based aggregation + SGM
    "c3": (2000, 3000, 256, "tower+cbca+sgm"),
    # the north-star size through the reference's whole GPU path (+ the build-defined CBCA)
    "north_star_sgm": (1024, 1024, 192, "tower+cbca+sgm"),
    # the cones pair through the same path (plumbing-size case of the SGM workloads)
    "cones_sgm": (375, 450, 64, "tower+cbca+sgm"),
    # BASELINE config 4: Middlebury-2005/2006 scale pairs, one pair per GPU (pair-DP)
    "c4": (1110, 1390, 256, "tower+cv_wta"),
    # BASELINE config 5: one 4K pair, D = 512 (the fused CV+WTA never materialises the 17 GB volume, so
    # N = 1 fits one GPU; N > 1 shards it by disparity block)
    "c5": (2160, 3840, 512, "tower+cv_wta"),
}
REF_GPU_PATH_MAX_VOX = 1110 * 1390 * 256   # stages.reference_gpu_path (L/R volumes + S resident) up to C4
CBCA_ITERS, CBCA_L1, CBCA_TAU = 2, 14, 0.02
PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: fp32 matrix (= vector) peak
PEAK_BF16_TFLOPS = 2516.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA (256 CU x 4 SIMD x 1024 flop/clk x 2.4 GHz)
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec peak
PEAK_VALU_PK_F32_OPS = 78.6   # T ops/s: 256 CUs x 64 lanes x 2 (v_pk_mul/add_f32) x 2.4 GHz, unfused
PEAK_VALU_F32_TOPS = 78.6     # non-fused f32 ops/s (one op per lane-slot; FMA counts 2 in the 157.3)
NF = 64
NLAYERS = 5


def measured_traffic(workload):
    """HBM bytes per launch of this workload's dominant kernel, from the newest committed PMC summary
    (profiles/rNN/traffic.json, written by tools/pmc_traffic.py from rocprofv3 FETCH_SIZE / WRITE_SIZE)."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "traffic.json")), reverse=True):
        try:
            entry = json.load(open(f)).get(workload)
        except (OSError, ValueError):
            continue
        if entry:
            return entry["traffic_bytes"], os.path.relpath(f, ROOT)
    return None, None


def conv_flops(hout, wout):
    return 2.0 * hout * wout * NF * 9 * NF


class Timer:
    """HIP events on torch's current stream (the stream every libsde launch uses)."""

    def __init__(self):
        self.pairs = []

    def start(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    def stop(self, e0):
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        self.pairs.append((e0, e1))

    def mean_ms(self):
        torch.cuda.synchronize()
        if not self.pairs:
            return float("nan")
        return float(np.mean([a.elapsed_time(b) for a, b in self.pairs]))

    def reset(self):
        self.pairs = []


TOWER_ARITH = {
    "fp32": "fp32 MFMA",
    "bf16x6": "bf16x6: fp32 operands split exactly into 3 bf16 parts, 6 leading partial products on bf16 MFMA, "
              "fp32 accumulation (fp32-level error)",
    "f16x3": "f16x3: fp32 operands scaled by powers of two and split exactly into 2 fp16 parts, 3 leading partial "
             "products on f16 MFMA, fp32 accumulation (~2^-22 per product; fp32-level error, checked vs the fp32 "
             "MFMA tower in stages)",
    "f16x3m32": "f16x3 arithmetic with layers 3..L on the v_mfma_f32_32x32x16_f16 direct kernel (the default f16x3 "
                "runs them on v_mfma_f32_16x16x32_f16)",
    "f16x3w": "f16x3 arithmetic with Winograd F(2x2,3x3) for layers 3..L: V = B^T d B in fp32 split into 2 fp16 "
              "parts, U = G g G^T formed in fp64 on the host and split, 3 partial products per Winograd product "
              "(2.25x fewer than direct), fp32 accumulation and output transform (fp32-level error)",
}


def make_step(m: StereoMatcher, what: str, t_conv: Timer, t_cv: Timer, t_tower: Timer):
    """One pass of the hot path.  The tower runs through the shipped StereoMatcher.features with a
    launch hook (pipeline.tower_steps: the same launches and bits as the one-call
    sde_tower_forward_batch, checked in main), so single kernels can be timed."""
    if what == "tower+cbca+sgm":
        def step_sgm(timed=None):
            e = t_tower.start() if timed == "stages" else None
            m.features()
            if e is not None:
                t_tower.stop(e)
            e = t_cv.start() if timed == "stages" else None
            out = m.sgm_path(post=True)
            if e is not None:
                t_cv.stop(e)
            return out
        return step_sgm

    def conv_hook(layer, launch):
        e = t_conv.start() if layer == 3 else None
        launch()
        if e is not None:
            t_conv.stop(e)

    def step(timed=None):
        """timed: None (warm-up), "conv" (the timed region: HIP events around the roofline kernel
        only) or "stages" (after the timed region: events around the tower and the CV+WTA)."""
        if what == "tower+cv_wta":
            e_t = t_tower.start() if timed == "stages" else None
            m.features(on_launch=conv_hook if timed == "conv" else (lambda layer, launch: launch()))
            if e_t is not None:
                t_tower.stop(e_t)
        e = t_cv.start() if timed == "stages" else None
        m.cost_wta()
        if e is not None:
            t_cv.stop(e)
        return m.disp

    return step


def cpu_share():
    """Host threads the CPU baseline may use: OMP_NUM_THREADS when the launcher sets it (16 on a one-GPU
    box), else min(16, cpu_count)."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, n if n > 0 else min(16, os.cpu_count() or 1))


def cpu_baseline(H, W, D, what, budget_s=15.0):
    """The C oracle (exact) on a bounded sample of the same workload: one thread, then the host's CPU
    share (min(16, cpu_count): row bands on Python threads for the tower + CV/WTA path, OpenMP over
    scanlines for the SGM path)."""
    import oracle
    from scenedepthestimation_amd import mc_cnn
    oracle.build()
    oracle.set_threads(1)
    # the box's CPU share: one GPU's box allots 16 host CPUs (OMP_NUM_THREADS=16 there), while
    # os.cpu_count() reports the whole host's (256 on the MI355X boxes): more threads would contend
    # with other jobs' shares rather than measure this port
    nt = cpu_share()
    left, right, _ = stereo_pair(H, W, D, seed=0)
    w = mc_cnn.synthetic_weights(NLAYERS)
    hw, hb = mc_cnn.layer_lists(w, NLAYERS)

    def run(rows):
        t0 = time.perf_counter()
        if what == "tower+cv_wta":
            feats = []
            for img in (left, right):
                pad = oracle.pad_image(oracle.znorm(img.astype(np.float32)), 2 * NLAYERS + 1)
                feats.append(oracle.tower_forward(pad[:rows + 2 * NLAYERS], hw, hb))
            fl, fr = feats
        else:
            from scenedepthestimation_amd.synthetic import features
            fl, fr = features(rows, W, seed=0), features(rows, W, seed=1)
            t0 = time.perf_counter()
        oracle.cv_wta_shard(fl, fr, 0, D)
        return time.perf_counter() - t0

    if what == "tower+cbca+sgm":
        # SGM's vertical and diagonal paths need whole columns: time a crop of the same workload
        # (rows x cols of the same pair, full D) through tower + L/R cost volume + CBCA + 8-path SGM
        # (both sides) + WTA + LR check + LRC + median, and scale per voxel.
        def run_crop(hc, wc):
            t0 = time.perf_counter()
            feats, zs = [], []
            for img in (left, right):
                crop = img[:hc, :wc]
                z = oracle.znorm(crop.astype(np.float32))
                zs.append(z)
                feats.append(oracle.tower_forward(oracle.pad_image(z, 2 * NLAYERS + 1), hw, hb))
            cl, cr = oracle.cost_volume_hwd(feats[0], feats[1], D, invalid=1.0, right=True)
            al, ar = oracle.cbca_arms(zs[0], CBCA_L1, CBCA_TAU), oracle.cbca_arms(zs[1], CBCA_L1, CBCA_TAU)
            cl, cr = oracle.cbca_lr(cl, cr, al, ar, CBCA_ITERS, L1=CBCA_L1)
            dl = oracle.wta_sgm(oracle.sgm_8path(cl, oracle.sgm_penalties(left[:hc, :wc])))
            dr = oracle.wta_sgm(oracle.sgm_8path(cr, oracle.sgm_penalties(right[:hc, :wc])))
            a, _ = oracle.lr_check(dl, dr)
            oracle.median5(oracle.lrc_fill(dl, a), dl)
            return time.perf_counter() - t0
        oracle.set_threads(nt)
        hc, wc = 16, max(D + 16, 64)
        t1 = run_crop(hc, wc)
        hc = int(max(16, min(H, hc * budget_s / max(t1, 1e-6))))
        t = run_crop(hc, wc)
        oracle.set_threads(1)
        return {"value": hc * wc * D / t / 1e6, "unit": "Mpixel-disparities/s", "cores": nt, "kind": "port",
                "sample": f"{hc} x {wc} crop x D={D} of the {H}x{W} pair through the full GPU path restated in C "
                          f"(fp64 tower, L/R cost volume, CBCA x{CBCA_ITERS}, 8-path SGM both sides, WTA, LR check, "
                          f"LRC, median), OpenMP over scanlines on {nt} threads, {t:.1f} s"}
    t1 = run(1)
    rows = int(max(1, min(H, budget_s / max(t1, 1e-6))))
    t = run(rows)
    single = rows * W * D / t / 1e6
    desc = (f"({what}, exact C restatement, {'fp64 tower + ' if what == 'tower+cv_wta' else ''}pairwise-f32 cost "
            f"+ WTA1)")
    # the same restatement on the host's CPU share (ctypes releases the GIL: one row band per thread)
    if what == "tower+cv_wta" and nt > 1:
        import concurrent.futures as cf
        rows_mt = int(min(H, rows * nt))
        bands = [(i * rows_mt // nt, (i + 1) * rows_mt // nt) for i in range(nt)]

        def band(r0, r1):
            feats = []
            for img in (left, right):
                pad = oracle.pad_image(oracle.znorm(img.astype(np.float32)), 2 * NLAYERS + 1)
                feats.append(oracle.tower_forward(pad[r0:r1 + 2 * NLAYERS], hw, hb))
            oracle.cv_wta_shard(feats[0], feats[1], 0, D)
        t0 = time.perf_counter()
        with cf.ThreadPoolExecutor(nt) as ex:
            list(ex.map(lambda b: band(*b), bands))
        tm = time.perf_counter() - t0
        return {"value": rows_mt * W * D / tm / 1e6, "unit": "Mpixel-disparities/s", "cores": nt, "kind": "port",
                "sample": f"{rows_mt} of {H} rows x {W} cols x D={D} {desc}, {nt} threads (one row band each), "
                          f"{tm:.1f} s wall",
                "single_thread": {"value": single, "cores": 1, "sample": f"{rows} rows, {t:.1f} s"}}
    return {"value": single, "unit": "Mpixel-disparities/s", "cores": 1, "kind": "port",
            "sample": f"{rows} of {H} rows x {W} cols x D={D} {desc}, {t:.1f} s"}


def numpy_baseline(H, W, D, budget_s=8.0):
    """The NumPy restatement of the reference's CPU path (oracle/np_restatement.py: the same
    np.multiply / np.sum expressions as process_functional.py:48-73, which is what
    match_single.py:51-53 runs), single-threaded, on bounded row samples of the workload's features
    (given; the tower is not in these figures).  WTA1 (process_functional.py:96-113) is timed two
    ways and labelled apart: the reference's own per-pixel Python loop ("reference_loop_wta1": the
    CPU path as it actually runs) and np.argmin ("argmin_wta1": a vectorised restatement, several
    times faster than what the reference runs)."""
    from oracle.np_restatement import compute_cost_volume_np, wta1_loop, wta1_np
    from scenedepthestimation_amd.synthetic import features

    def sample(rows):
        return features(rows, W, seed=0), features(rows, W, seed=1)

    def run_cv(rows):
        fl, fr = sample(rows)
        t0 = time.perf_counter()
        cv = compute_cost_volume_np(fl, fr, D)
        t1 = time.perf_counter()
        wta1_np(cv)
        return t1 - t0, time.perf_counter() - t1, cv
    tc, ta, _ = run_cv(2)
    rows = int(max(1, min(H, budget_s / max((tc + ta) / 2, 1e-6))))
    tc, ta, cv = run_cv(rows)
    # the Python loop on whole rows of the same volume (~W * D scalar steps each), for >= 1 s
    t0 = time.perf_counter()
    nrows = 0
    while nrows < cv.shape[1] and (nrows == 0 or time.perf_counter() - t0 < 1.0):
        wta1_loop(cv[:, nrows:nrows + 1])
        nrows += 1
    tl = (time.perf_counter() - t0) / nrows
    vox = float(W) * D
    per_cv, per_arg, per_loop = tc / (rows * vox), ta / (rows * vox), tl / vox     # seconds per voxel
    return {"value": 1e-6 / (per_cv + per_arg), "unit": "Mpixel-disparities/s", "cores": 1, "kind": "port",
            "what": "compute_cost_volume (NumPy) + WTA1 as np.argmin -- vectorised, NOT the reference's loop",
            "reference_loop_wta1": {
                "value": 1e-6 / (per_cv + per_loop), "unit": "Mpixel-disparities/s", "cores": 1,
                "what": "compute_cost_volume (NumPy) + WTA1 as the reference's per-pixel Python loop "
                        "(process_functional.py:96-113): the CPU path match_single.py:51-53 runs",
                "ms_per_pair_estimate": (per_cv + per_loop) * H * W * D * 1e3,
                "sample": f"loop timed on {nrows} row(s) x {W} cols x D={D} ({tl * nrows:.2f} s)"},
            "argmin_wta1_share": per_arg / (per_cv + per_arg),
            "sample": f"{rows} of {H} rows x {W} cols x D={D}: compute_cost_volume {tc:.1f} s + np.argmin {ta:.1f} s, "
                      f"features given"}


def _events_ms(fn, reps=3):
    """Mean HIP-event time of fn() on torch's current stream over `reps` calls (after one warm call)."""
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def gpu_path_stages(m: StereoMatcher, prefix: str = ""):
    """The reference's GPU path (disparity_compute_by_gpu, process_functional.py:1093-1267, + the
    build-defined CBCA) on m's resident features: whole-path time and the HBM fraction of each
    cost-volume / aggregation kernel on SURVEY.md sec. 8(d)'s algorithmic bytes (north_star's
    "cost-volume + aggregation kernels"), each launch timed alone with HIP events."""
    H, W, D = m.H, m.W, m.D
    vox = float(H) * W * D
    b = m.sgm_bufs
    out = {}
    path_ms = _events_ms(lambda: m.sgm_path(post=True))
    tower_ms = _events_ms(lambda: m.features())
    out[prefix + "gpu_path_ms"] = path_ms
    # the SGM volumes' placement draws (pipeline.StereoMatcher._place_sgm_volumes): pair ms per draw
    out[prefix + "sgm_placement_draws_ms"] = m.sgm_placement_ms
    out[prefix + "ms_per_pair_tower_plus_gpu_path"] = tower_ms + path_ms
    kern = {}
    # cvlr3_kernel: reads both feature maps once, writes the L and R [H,W,D] volumes -- the left one only
    # when the aggregation follows (sde_cbca_lr writes the right one as the aggregated left one's shear)
    both = m.cbca_iters <= 0
    ms = _events_ms(lambda: ops.cost_volume(m.feat[0], m.feat[1], D, layout="HWD", right=both, invalid=1.0,
                                            out_left=b["cv"][0], out_right=b["cv"][1] if both else None))
    cvlr_ms = ms
    kern["cvlr3_kernel (" + ("L/R volumes)" if both else "L volume)")] = \
        (ms, 4.0 * H * W * (2 * NF + (2 if both else 1) * D))
    if m.cbca_iters > 0:
        # sde_cbca_lr (definition v2): the left volume's iterations, each a horizontal and a vertical
        # pass reading + writing 4 B per valid voxel, then the shear into the right volume (4 + 4 B per
        # valid voxel); valid = right-image pixel inside the image, sum_d H * max(W - d, 0) voxels
        valid = float(H) * sum(max(W - d, 0) for d in range(D))
        ms = _events_ms(lambda: ops.cbca_lr(b["cv"][0], b["cv"][1], b["arms"][0], b["arms"][1], m.cbca_L1,
                                            m.cbca_iters, tmp=b["S"][0], workspace=b["cbca_ws"]))
        kern[f"cbca_h/v_kernel + cbca_rotate_kernel ({m.cbca_iters} iterations, one volume + shear)"] = \
            (ms, (16.0 * m.cbca_iters + 8.0) * valid)
    ms = _events_ms(lambda: ops.sgm_8path_wta_pair(b["cv"][0], b["pen"][0], b["S"][0], b["disp"][0], b["cv"][1],
                                                   b["pen"][1], b["S"][1], b["disp"][1], zero_du_penalties=True))
    # per side: UD+DU 8 B/voxel, five passes 12 B, DU-RL + WTA 8 B, + 4 B/pixel of disparity
    kern["sgm_scan_kernel (8 paths + WTA, both sides, 7 launches)"] = (ms, 2 * (76.0 * vox + 4.0 * H * W))
    per = {}
    tb = tt = 0.0
    tkeys = {"cvlr": "cvlr", "cbca": "cbca_lr", "sgm_": "sgm_pair"}
    for k, (ms, byt) in kern.items():
        gbs = byt / (ms * 1e-3) / 1e9
        per[k] = {"ms": ms, "GB": byt / 1e9, "GB_s": gbs, "hbm_frac": gbs / PEAK_HBM_GBS}
        # PMC HBM bytes of the same launch(es) at 1024^2 x 192 (profiles/rNN/traffic.json)
        tk = next(v for a, v in tkeys.items() if k.startswith(a))
        tr, src = measured_traffic(tk) if (H, W, D) == (1024, 1024, 192) else (None, None)
        if tr is not None:
            per[k]["traffic_GB"] = tr / 1e9
            per[k]["traffic_source"] = src
        tb += byt
        tt += ms
    # the L/R volume kernel's other bound: every valid voxel is NumPy's exact fp32 dot product, 64
    # separately rounded products + 64 adds (pairwise tree, 0.0 + s), on the packed-fp32 VALU
    k0 = next(iter(per))
    per[k0]["valu_ops"] = 128.0 * vox
    per[k0]["valu_frac"] = 128.0 * vox / (cvlr_ms * 1e-3) / (PEAK_VALU_PK_F32_OPS * 1e12)
    per[k0]["valu_peak"] = f"{PEAK_VALU_PK_F32_OPS} T separately rounded fp32 ops/s (256 CU x 64 lanes x 2 packed x 2.4 GHz)"
    out[prefix + "cv_aggregation_kernels"] = per
    out[prefix + "cv_aggregation_aggregate"] = {
        "ms": tt, "GB": tb / 1e9, "GB_s": tb / (tt * 1e-3) / 1e9, "hbm_frac": tb / (tt * 1e-3) / 1e9 / PEAK_HBM_GBS,
        "what": f"cvlr + CBCA ({m.cbca_iters} iterations, sde_cbca_lr) + SGM pair on sec. 8(d) algorithmic bytes"}
    return out


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def resolve_mode(mode, world, what):
    """--mode auto -> the scheme that runs: one GPU: the single-device hot path (pairdp); N > 1 on the
    tower + CV/WTA workloads: north_star's disparity-sharded cost volume (dshard, strong scaling), with the
    other schemes timed beside it in stages.multi_gpu_modes; the SGM workloads (every disparity per step)
    run pair-DP replicas.  An explicit sharded mode on an SGM workload at N > 1 is refused."""
    if mode == "auto":
        return "dshard" if world > 1 and what == "tower+cv_wta" else "pairdp"
    if world > 1 and what != "tower+cv_wta" and mode != "pairdp":
        raise SystemExit(f"--mode {mode}: the sharded schemes run the tower + CV/WTA workloads only "
                         f"(SGM needs every disparity per step: replicas only, --mode pairdp)")
    return mode


def c3_stage(args, steps=3):
    """BASELINE config 3 on the north-star line: the 2000x3000 pair at D = 256 through
    tower x2 + L volume + CBCA x2 (sde_cbca_lr) + SGM both sides + WTA + LR check / LRC / median
    (disparity_compute_by_gpu, process_functional.py:1093-1267), `steps` timed steps after one warm-up with
    the barrier-free single-GPU clock of the main line (synchronise, wall clock, synchronise), plus the per-kernel
    HBM fractions of gpu_path_stages.  No CPU leg."""
    H, W, D, what = WORKLOADS["c3"]
    m = StereoMatcher(H, W, D, tower_precision=args.tower_precision, sgm=True, cbca_iters=CBCA_ITERS,
                      cbca_L1=CBCA_L1, cbca_tau=CBCA_TAU)
    left, right, _ = stereo_pair(H, W, D, seed=0)
    m.load_images(left, right)
    t = Timer()
    step = make_step(m, what, t, t, t)
    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    vox = float(H) * W * D
    out = {"workload": "c3", "H": H, "W": W, "D": D, "steps": steps, "ms_per_pair": el / steps * 1e3,
           "Mvox_s": vox * steps / el / 1e6,
           "pipeline": "u8 pair -> preprocess -> tower x2 -> L volume -> CBCA x2 (+ shear) -> SGM both sides + WTA "
                       "-> LR check / LRC / median"}
    out.update(gpu_path_stages(m))
    del m
    torch.cuda.empty_cache()
    return out


def make_mode(mode, H, W, D, what, rank, world, args, t_conv, t_cv, t_tower):
    """-> (step, pairs_per_step, scaling, parallelism, result): one multi-GPU scheme (or the single-device
    path, pairdp) on this rank.  The strong-scaling schemes match ONE pair (seed 0 on every rank); pair-DP
    matches its own pair per rank (seed = rank).  result() returns the disparity map the last step made
    (rank 0's pair for pair-DP)."""
    if mode == "pairdp" or world == 1:
        sgm = what == "tower+cbca+sgm"
        m = StereoMatcher(H, W, D, tower_precision=args.tower_precision, cv_mode=args.cv_mode, sgm=sgm,
                          cbca_iters=CBCA_ITERS if sgm else 0, cbca_L1=CBCA_L1, cbca_tau=CBCA_TAU)
        left, right, _ = stereo_pair(H, W, D, seed=rank)
        m.load_images(left, right)
        if what == "cv_wta":
            m.features()
        step = make_step(m, what, t_conv, t_cv, t_tower)
        step.matcher = m
        res = (lambda: m.sgm_bufs["disp"][0]) if sgm else (lambda: m.disp)
        return step, world, "weak", f"pairdp{world}", res
    left, right, _ = stereo_pair(H, W, D, seed=0)
    if mode == "dshard":
        obj = DisparityShardedMatcher(H, W, D, rank, world, tower_precision=args.tower_precision)
        obj.m.load_images(left, right)
    elif mode == "dshard_rep":
        obj = ReplicatedDisparityShardedMatcher(H, W, D, rank, world, tower_precision=args.tower_precision)
        obj.load_images(left, right)
    elif mode == "rowband":
        obj = RowBandMatcher(H, W, D, rank, world, tower_precision=args.tower_precision, cv_mode=args.cv_mode)
        obj.load_images(left, right)
    else:
        raise ValueError(mode)

    def step(timed=None):
        e = t_tower.start() if timed == "stages" else None
        r = obj.match()
        if e is not None:
            t_tower.stop(e)
        return r
    return step, 1, "strong", f"{mode}{world}", lambda: obj.disp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)     # ~0.1 s timed at the north star: 10 steps (20 ms) swung 2.05-2.25 ms/pair box to box
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--workload", default="north_star", choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="auto", choices=["auto", "pairdp", "dshard", "dshard_rep", "rowband"])
    ap.add_argument("--dump-disp", default=None, help="rank 0 saves the disparity map (.npy; auto mode: also "
                                                         "<path>.<mode>.npy for every other scheme)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c3", action="store_true", help="north_star: skip stages.c3 (BASELINE config 3 timed "
                                                         "beside the line)")
    ap.add_argument("--tower-precision", default="f16x3", choices=["fp32", "bf16x6", "f16x3", "f16x3w", "f16x3m32"])
    ap.add_argument("--cv-mode", default="certified", choices=["certified", "exact"])
    args = ap.parse_args()

    rank, world, local = init_from_env()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # (init_from_env selected the device: cuda:LOCAL_RANK, or LOCAL_RANK mod the device count for
    # ranks sharing a GPU over gloo)
    H, W, D, what = WORKLOADS[args.workload]
    left, right, _ = stereo_pair(H, W, D, seed=rank)     # this rank's pair (pair-DP; rank 0: seed 0)
    mode = resolve_mode(args.mode, world, what)

    t_conv, t_cv, t_tower = Timer(), Timer(), Timer()
    m = None
    step, pairs_per_step, scaling, par, result = make_mode(mode, H, W, D, what, rank, world, args,
                                                           t_conv, t_cv, t_tower)
    if mode == "pairdp":
        m = step.matcher

    def timed_run(step_fn, nsteps, nwarm, timed):
        for _ in range(nwarm):
            step_fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(nsteps):
            step_fn(timed=timed)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        # max over ranks (gloo reduces host tensors: SDE_DIST_BACKEND=gloo runs ranks on a shared GPU)
        tt = torch.tensor([el], dtype=torch.float64,
                          device="cuda" if world == 1 or dist.get_backend() == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    elapsed = timed_run(step, args.steps, args.warmup, "conv")
    # per-stage times from a few extra steps outside the timed region (their events would add
    # stream barriers to the timed steps)
    for _ in range(min(args.steps, 5)):
        step(timed="stages")
    torch.cuda.synchronize()
    disp_primary = result().detach().clone() if args.dump_disp else None

    multi = None
    if world > 1 and args.mode == "auto" and what == "tower+cv_wta":
        # the other multi-GPU schemes on the same pair, same ranks, same clock discipline (barrier +
        # max over ranks); pair-DP is weak scaling (world pairs per step), the rest strong (one pair)
        multi = {mode: {"ms_per_step": elapsed / args.steps * 1e3, "pairs_per_step": pairs_per_step,
                        "scaling": scaling, "primary": True}}
        others = [x for x in ("dshard", "dshard_rep", "rowband", "pairdp") if x != mode]
        del step
        torch.cuda.empty_cache()
        for om in others:
            st2, pps2, sc2, _par2, res2 = make_mode(om, H, W, D, what, rank, world, args, Timer(), Timer(), Timer())
            n2 = min(args.steps, 10)
            el2 = timed_run(st2, n2, min(args.warmup, 3), None)
            multi[om] = {"ms_per_step": el2 / n2 * 1e3, "pairs_per_step": pps2, "scaling": sc2,
                         "Mvox_s": float(H) * W * D * pps2 * n2 / el2 / 1e6}
            if args.dump_disp and rank == 0:
                np.save(f"{args.dump_disp}.{om}.npy", res2().cpu().numpy())
            del st2, res2
            torch.cuda.empty_cache()
    if args.dump_disp and rank == 0:
        np.save(args.dump_disp, disp_primary.cpu().numpy())

    vox = float(H) * W * D
    value = vox * pairs_per_step * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    roof = None
    parity = None
    host_io_ms = None
    stages = {}
    if what == "tower+cbca+sgm" and mode == "pairdp":
        stages["tower_ms_pair"] = t_tower.mean_ms()
        stages["gpu_path_ms"] = t_cv.mean_ms()
        tim = {}
        m.sgm_path(post=True, timings=tim)           # one synchronised pass, per-stage wall times
        stages.update({f"{k}_ms": v * 1e3 for k, v in tim.items()})
        g = gpu_path_stages(m)
        stages.update(g)
        sgm_ms, sgm_bytes = None, 2 * (76.0 * vox + 4.0 * H * W)
        for k, v in g["cv_aggregation_kernels"].items():
            if k.startswith("sgm"):
                sgm_ms = v["ms"]
            if k.startswith("cbca"):
                stages["cbca_lr_ms"] = v["ms"]
                stages["cbca_lr_hbm_GBs"] = v["GB_s"]
        stages["sgm_pair_ms"] = sgm_ms
        ach = sgm_bytes / (sgm_ms * 1e-3) / 1e9
        roof = {"kernel": "sgm_scan_kernel (8-path SGM + WTA, both sides, 7 launches: DU folded into UD, WTA "
                          "into DU-RL)", "bound": "hbm",
                "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                "traffic": None,
                "per_launch": f"2 sides x (8 + 5 x 12 + 8) B/voxel x {vox / 1e6:.0f} Mvox + disp = "
                              f"{sgm_bytes / 1e9:.2f} GB over {sgm_ms:.3f} ms (7 launches)"}
    elif mode == "pairdp":
        cv_ms = t_cv.mean_ms()
        bytes_cv = 4.0 * H * W * 2 * NF + 4.0 * H * W
        stages["cv_wta_ms"] = cv_ms
        stages["cv_wta_hbm_GBs"] = bytes_cv / (cv_ms * 1e-3) / 1e9
        if args.cv_mode == "exact":   # 127 separately rounded f32 ops per voxel on VALU
            stages["cv_wta_valu_Tops"] = 127.0 * vox / (cv_ms * 1e-3) / 1e12
            stages["cv_wta_valu_frac"] = stages["cv_wta_valu_Tops"] / PEAK_VALU_F32_TOPS
        stages["cv_wta_Mvox_s"] = vox / (cv_ms * 1e-3) / 1e6
        stages["cv_mode"] = args.cv_mode
        if args.cv_mode == "certified":
            stages["cv_exact_fixup_pixels"] = ops.cv_wta_fixups(m.cv_ws)
        if what == "tower+cv_wta":
            conv_ms = t_conv.mean_ms()
            hout = H + 2 * (NLAYERS - 3)
            wout = W + 2 * (NLAYERS - 3)
            fl = 2 * conv_flops(hout, wout)   # one launch = both images of the pair
            stages["tower_ms_pair"] = t_tower.mean_ms()
            stages["conv_layer3_ms"] = conv_ms
            stages["conv_fp32_equiv_TFLOPs"] = fl / (conv_ms * 1e-3) / 1e12
            if m.tower_precision in ("bf16x6", "f16x3", "f16x3w", "f16x3m32"):
                # 6 bf16 / 3 f16 partial products per fp32 product: the roof is the dense bf16/f16 MFMA rate
                # (Winograd: 3 per Winograd product, 16 per 2x2 outputs instead of 36)
                k, kt = (6, "bf16") if m.tower_precision == "bf16x6" else (3, "f16")
                if m.tower_precision == "f16x3w":
                    k = 3 * 16 / 36
                ach = k * fl / (conv_ms * 1e-3) / 1e12
                kname = ("wino_kernel<false,true,true>" if m.tower_precision == "f16x3w" else
                         "conv64_h16_kernel<false,true,true,false,false,false,false>" if m.tower_precision == "f16x3" else
                         f"conv64_x6p_kernel<false,false,true,true,{str(kt == 'f16').lower()}>")
                roof = {"kernel": f"{kname} (tower layer 3, {m.tower_precision})", "bound": "mfma",
                        "achieved": ach, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_BF16_TFLOPS,
                        "traffic": None,
                        "per_launch": f"{k:.4g} x {fl / 1e9:.2f} GFLOP {kt} (2 images x 2*{hout}*{wout}*64*576 fp32-equivalent) "
                                      f"over {conv_ms:.3f} ms"}
            else:
                ach = fl / (conv_ms * 1e-3) / 1e12
                roof = {"kernel": "conv64_mfma_kernel<false,false> (tower layer 3, fp32)", "bound": "mfma",
                        "achieved": ach, "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_FP32_TFLOPS,
                        "traffic": None,
                        "per_launch": f"{fl / 1e9:.2f} GFLOP = 2 images x 2*{hout}*{wout}*64*576 over {conv_ms:.3f} ms"}
            if m.tower_precision != "fp32":
                # the same features through the fp32-MFMA tower: max |difference| on this very image
                ref = torch.empty_like(m.feat[0])
                ops.tower_forward(m.img_pad[0], m.packed, NLAYERS, NF, out=ref, workspace=m.ws, precision="fp32")
                ops.tower_forward(m.img_pad[0], m.packed, NLAYERS, NF, out=m.feat[0], workspace=m.ws,
                                  precision=m.tower_precision)
                stages[f"tower_{m.tower_precision}_vs_fp32_max_abs"] = float((ref - m.feat[0]).abs().max().item())
            # the reference's boundary hands over host arrays (host u8 images in ->
            # disparity out): pinned host buffers, async copies on the stream, one synchronisation per
            # pair; reported beside `value` (resident inputs), never as it
            hl = torch.from_numpy(np.ascontiguousarray(left)).pin_memory()
            hr = torch.from_numpy(np.ascontiguousarray(right)).pin_memory()
            hd = torch.empty((H, W), dtype=torch.float32).pin_memory()
            st = torch.cuda.current_stream()

            def host_pair():
                m.img_u8[0].copy_(hl, non_blocking=True)
                m.img_u8[1].copy_(hr, non_blocking=True)
                hd.copy_(m.match(), non_blocking=True)
                st.synchronize()
            for _ in range(2):
                host_pair()
            t0 = time.perf_counter()
            for _ in range(10):
                host_pair()
            host_io_ms = (time.perf_counter() - t0) / 10 * 1e3
            stages["ms_per_pair_host_io"] = host_io_ms
            # the same boundary over a stream of pairs: pair i+1's images go up and pair i-1's map comes down on
            # a copy stream while pair i computes (two pinned / device staging sets; events order each copy
            # against the compute that produces or consumes it).  Per pair amortised over 10 pairs.
            cs = torch.cuda.Stream()
            n_pipe = 10
            hin = [(torch.from_numpy(np.ascontiguousarray(left)).pin_memory(),
                    torch.from_numpy(np.ascontiguousarray(right)).pin_memory()) for _ in range(2)]
            hout = [torch.empty((H, W), dtype=torch.float32).pin_memory() for _ in range(2)]
            din = [(torch.empty_like(m.img_u8[0]), torch.empty_like(m.img_u8[1])) for _ in range(2)]
            dout = [torch.empty((H, W), dtype=torch.float32, device=m.device) for _ in range(2)]

            def pipelined(n):
                up = [torch.cuda.Event() for _ in range(n)]
                done = [torch.cuda.Event() for _ in range(n)]
                freed = [torch.cuda.Event() for _ in range(n)]   # staging input slot read by the compute
                down = [torch.cuda.Event() for _ in range(n)]    # staging output slot read by the D2H copy
                with torch.cuda.stream(cs):
                    din[0][0].copy_(hin[0][0], non_blocking=True)
                    din[0][1].copy_(hin[0][1], non_blocking=True)
                    up[0].record(cs)
                for i in range(n):
                    k = i & 1
                    if i + 1 < n:   # the next pair's images, into the other slot once pair i-1 consumed it
                        with torch.cuda.stream(cs):
                            if i >= 1:
                                cs.wait_event(freed[i - 1])
                            din[k ^ 1][0].copy_(hin[k ^ 1][0], non_blocking=True)
                            din[k ^ 1][1].copy_(hin[k ^ 1][1], non_blocking=True)
                            up[i + 1].record(cs)
                    st.wait_event(up[i])
                    m.img_u8[0].copy_(din[k][0], non_blocking=True)
                    m.img_u8[1].copy_(din[k][1], non_blocking=True)
                    freed[i].record(st)
                    if i >= 2:
                        st.wait_event(down[i - 2])
                    dout[k].copy_(m.match(), non_blocking=True)
                    done[i].record(st)
                    with torch.cuda.stream(cs):   # pair i's map down while pair i+1 computes
                        cs.wait_event(done[i])
                        hout[k].copy_(dout[k], non_blocking=True)
                        down[i].record(cs)
                cs.synchronize()
                st.synchronize()
            pipelined(2)
            t0 = time.perf_counter()
            pipelined(n_pipe)
            stages["ms_per_pair_host_io_pipelined"] = (time.perf_counter() - t0) / n_pipe * 1e3
            if not torch.equal(hout[(n_pipe - 1) & 1], hd):
                raise SystemExit("pipelined host-I/O pairs: disparity map differs from the per-pair path")
            # parity, outside the timed region: (1) the hooked layer-by-layer tower the timed steps ran
            # == the one-call sde_tower_forward_batch; (2) the certified map == the exact kernel's
            # over every pixel (and the minimum costs bit for bit)
            m.features(on_launch=lambda layer, launch: launch())
            hooked = m.feat2.clone()
            m.features()
            same_feat = bool(torch.equal(hooked, m.feat2))
            cert_disp, cert_min, _ = ops.cv_wta(m.feat[0], m.feat[1], 0, D, want=("disp", "min"), mode="certified",
                                                workspace=m.cv_ws)
            ex_disp, ex_min, _ = ops.cv_wta(m.feat[0], m.feat[1], 0, D, want=("disp", "min"), mode="exact")
            same_disp = bool(torch.equal(cert_disp, ex_disp))
            same_min = bool(torch.equal(cert_min.view(torch.int32), ex_min.view(torch.int32)))
            parity = {"checked": True, "pixels": H * W,
                      "certified_vs_exact_disparity_identical": same_disp,
                      "certified_vs_exact_min_cost_bits_identical": same_min,
                      "tower_hooked_vs_one_call_identical": same_feat}
            if not (same_disp and same_min and same_feat):
                raise SystemExit(f"parity check failed: {parity}")
            del cert_disp, cert_min, ex_disp, ex_min, hooked
            # the reference's default GPU path at the same size (match_single.py:49 ->
            # disparity_compute_by_gpu), + the build-defined CBCA x2: north_star's own target
            if vox <= REF_GPU_PATH_MAX_VOX:
                ms_ = StereoMatcher(H, W, D, tower_precision=args.tower_precision, sgm=True, cbca_iters=CBCA_ITERS,
                                    cbca_L1=CBCA_L1, cbca_tau=CBCA_TAU)
                ms_.load_images(left, right)
                ms_.features()
                stages["reference_gpu_path"] = gpu_path_stages(ms_)
                del ms_
                torch.cuda.empty_cache()
            if args.workload == "north_star" and world == 1 and not args.no_c3:
                stages["c3"] = c3_stage(args)
        else:
            ach = bytes_cv / (cv_ms * 1e-3) / 1e9
            kname = ("cv_wta_row_kernel + cv_wta_fixup_kernel (certified fused cost volume + WTA)"
                     if args.cv_mode == "certified" else "cv64_kernel<LEFT,WTA> (exact fused cost volume + WTA)")
            extra = (f"; VALU {stages['cv_wta_valu_frac']:.2f} of {PEAK_VALU_F32_TOPS} Top/s"
                     if "cv_wta_valu_frac" in stages else "")
            roof = {"kernel": kname, "bound": "hbm",
                    "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                    "traffic": None,
                    "per_launch": f"{bytes_cv / 1e6:.1f} MB = 4*H*W*(2*64+1) over {cv_ms:.3f} ms" + extra}
    else:
        stages[f"{mode}_step_ms"] = t_tower.mean_ms()
    if multi is not None:
        stages["multi_gpu_modes"] = multi

    if roof is not None:
        tb, src = measured_traffic(args.workload)
        roof["traffic"] = tb
        roof["traffic_unit"] = "bytes per launch (HBM, PMC)"
        roof["traffic_source"] = src

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(H, W, D, what)
        cpu["cpu_model"] = cpu_model()
        cpu["host_cpus_visible"] = os.cpu_count()
        cpu["cores_rationale"] = ("the one-GPU box's CPU share (OMP_NUM_THREADS); os.cpu_count() counts the "
                                  "whole host, whose other CPUs belong to other GPUs' jobs")
        if what in ("tower+cv_wta", "cv_wta"):
            cpu["numpy_restatement"] = numpy_baseline(H, W, D)

    if rank == 0:
        line = {
            "metric": "Mpixel-disparities/sec (H*W*D cost voxels per second, end-to-end per pair)",
            "value": value, "unit": "Mpixel-disparities/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_step, "ms_per_pair": ms_step / pairs_per_step * world
            if scaling == "weak" else ms_step,
            "higher_is_better": True, "scaling": scaling, "vs_baseline": None, "dtype": "f32",
            "tower_arith": TOWER_ARITH[args.tower_precision],
            "data": "synthetic (seeded textured pair, band disparity field; synthetic He-normal tower weights)",
            "config": {"workload": args.workload, "H": H, "W": W, "D": D, "C": NF, "nlayers": NLAYERS,
                       "pipeline": what, "global_batch": pairs_per_step, "parallelism": par},
            "roofline": roof, "cpu_baseline": cpu, "stages": stages,
        }
        if parity is not None:
            line["parity"] = parity
        if host_io_ms is not None:
            line["ms_per_pair_host_io"] = host_io_ms
            line["ms_per_pair_host_io_pipelined"] = stages.get("ms_per_pair_host_io_pipelined")
            line["host_io"] = ("host u8 pair in -> host f32 disparity out per pair: pinned buffers, async H2D/D2H "
                               "copies on the compute stream, one synchronisation (SURVEY.md sec. 8(d)'s ms/pair); _pipelined: the "
                               "same over a stream of 10 pairs, the copies of the next / previous pair on a second "
                               "stream while a pair computes (maps checked equal)")
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
