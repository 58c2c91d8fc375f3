#!/usr/bin/env python
"""bench.py -- throughput of the stereo matching hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload north_star|cones|cv]
                    [--mode pairdp|dshard] [--no-cpu-baseline]

A step = one stereo pair through the hot path with inputs resident in HBM:
u8 images -> z-norm + pad -> MC-CNN-fast tower (5 fp32-MFMA conv layers) on both
images -> fused exact cost volume + WTA over D disparities -> float32 disparity.
Default workload: the north-star size 1024x1024, D = 192 (BASELINE.json).

N > 1 (one process per GPU under torchrun, RCCL):
  pairdp : every rank matches its own pair each step (config 4) -- weak scaling,
           no collective on the data path;
  dshard : one pair per step, disparity-sharded over the ranks with the feature
           row-band all-gather and the (min, argmin) all-gather (config 5) --
           strong scaling.

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
from scenedepthestimation_amd.parallel import DisparityShardedMatcher, init_from_env  # noqa: E402
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
}
CBCA_ITERS, CBCA_L1, CBCA_TAU = 2, 14, 0.02
PEAK_FP32_TFLOPS = 157.3      # MI355X_MICROARCH.md: fp32 matrix (= vector) peak
PEAK_BF16_TFLOPS = 2516.0     # MI355X_MICROARCH.md: ~2.5 PF dense bf16 MFMA (256 CU x 4 SIMD x 1024 flop/clk x 2.4 GHz)
PEAK_HBM_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E spec peak
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
}


def make_step(m: StereoMatcher, what: str, t_conv: Timer, t_cv: Timer, t_tower: Timer):
    """One pass of the hot path, launched layer by layer so single kernels can be timed."""
    L = m.nlayers
    H, W = m.H, m.W
    # activation ping-pong buffers for layers 3..L, both images (layer 2 output is (H+2(L-2)) x ...)
    acts = [torch.empty((2 * (H + 2 * (L - 2)) * (W + 2 * (L - 2)) * NF,), dtype=torch.float32, device=m.device)
            for _ in range(2)]
    # f16x3 bound words per image (what sde_tower_forward_batch keeps in its workspace)
    words = torch.zeros((2, L), dtype=torch.float32, device=m.device)
    batched = m.split is None

    def tower_pair(timed):
        """Preprocess both images, then the tower layer by layer with both images per launch
        (sde_tower_layer_batch = what sde_tower_forward_batch launches), layer 3 timed."""
        e_t = t_tower.start() if timed == "stages" else None
        ops.preprocess_u8_batch(m.img_u82, L, out=m.img_pad2, stats=m.stats2)
        if not batched:   # split planes requested: per-image launches
            m.features_from_padded()
            if e_t is not None:
                t_tower.stop(e_t)
            return
        # split arithmetics: intermediate activations in the c-block-major layout, as sde_tower_forward runs them
        cbl = m.tower_precision in ("bf16x6", "f16x3")
        if m.tower_precision == "f16x3":
            words.zero_()
            ops.absmax_batch(m.img_pad2, words)
        hin, win = H + 2 * L - 4, W + 2 * L - 4
        first_out = acts[0][: 2 * hin * win * NF].view(2, hin, win, NF) if L > 2 else m.feat2
        ops.tower_layer_batch(m.img_pad2, m.packed, L, 2, first_out, precision=m.tower_precision,
                              out_cblock=cbl and L > 2, in_absmax=words[:, 0:1],
                              out_absmax=words[:, 1:2] if L > 2 else None)
        cur = 0
        for layer in range(3, L + 1):
            if layer == L:
                o = m.feat2
            else:   # a contiguous prefix of the ping-pong buffer, viewed at this layer's size
                o = acts[cur ^ 1][: 2 * (hin - 2) * (win - 2) * NF].view(2, hin - 2, win - 2, NF)
            src = acts[cur][: 2 * hin * win * NF].view(2, hin, win, NF)
            e = t_conv.start() if (timed == "conv" and layer == 3) else None
            ops.tower_layer_batch(src, m.packed, L, layer, o, precision=m.tower_precision,
                                  in_cblock=cbl, out_cblock=cbl and layer < L, in_absmax=words[:, layer - 2:layer - 1],
                                  out_absmax=words[:, layer - 1:layer] if layer < L else None)
            if e is not None:
                t_conv.stop(e)
            hin, win = hin - 2, win - 2
            cur ^= 1
        if e_t is not None:
            t_tower.stop(e_t)
        m.split_valid = False

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

    def step(timed=None):
        """timed: None (warm-up), "conv" (the timed region: HIP events around the roofline kernel
        only) or "stages" (after the timed region: events around the tower and the CV+WTA)."""
        if what == "tower+cv_wta":
            tower_pair(timed)
        e = t_cv.start() if timed == "stages" else None
        m.cost_wta()
        if e is not None:
            t_cv.stop(e)
        return m.disp

    return step


def cpu_baseline(H, W, D, what, budget_s=15.0):
    """The C oracle (single thread, exact) on a bounded row band of the same workload."""
    import oracle
    from scenedepthestimation_amd import mc_cnn
    oracle.build()
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
            cl = oracle.cbca(cl, al, ar, "left", CBCA_ITERS)
            cr = oracle.cbca(cr, ar, al, "right", CBCA_ITERS)
            dl = oracle.wta_sgm(oracle.sgm_8path(cl, oracle.sgm_penalties(left[:hc, :wc])))
            dr = oracle.wta_sgm(oracle.sgm_8path(cr, oracle.sgm_penalties(right[:hc, :wc])))
            a, _ = oracle.lr_check(dl, dr)
            oracle.median5(oracle.lrc_fill(dl, a), dl)
            return time.perf_counter() - t0
        hc, wc = 16, max(D + 16, 64)
        t1 = run_crop(hc, wc)
        hc = int(max(16, min(H, hc * budget_s / max(t1, 1e-6))))
        t = run_crop(hc, wc)
        return {"value": hc * wc * D / t / 1e6, "unit": "Mpixel-disparities/s", "cores": 1, "kind": "port",
                "sample": f"{hc} x {wc} crop x D={D} of the {H}x{W} pair through the full GPU path restated in C "
                          f"(fp64 tower, L/R cost volume, CBCA x{CBCA_ITERS}, 8-path SGM both sides, WTA, LR check, "
                          f"LRC, median), {t:.1f} s"}
    t1 = run(1)
    rows = int(max(1, min(H, budget_s / max(t1, 1e-6))))
    t = run(rows)
    single = rows * W * D / t / 1e6
    desc = (f"({what}, exact C restatement, {'fp64 tower + ' if what == 'tower+cv_wta' else ''}pairwise-f32 cost "
            f"+ WTA1)")
    # the same restatement on the host's CPU share (ctypes releases the GIL: one row band per thread)
    nt = min(16, os.cpu_count() or 1)
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="north_star", choices=sorted(WORKLOADS))
    ap.add_argument("--mode", default="pairdp", choices=["pairdp", "dshard"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--tower-precision", default="f16x3", choices=["fp32", "bf16x6", "f16x3"])
    ap.add_argument("--cv-mode", default="certified", choices=["certified", "exact"])
    args = ap.parse_args()

    rank, world, local = init_from_env()
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    H, W, D, what = WORKLOADS[args.workload]
    left, right, _ = stereo_pair(H, W, D, seed=rank)

    t_conv, t_cv, t_tower = Timer(), Timer(), Timer()
    if args.mode == "dshard" and world > 1:
        dm = DisparityShardedMatcher(H, W, D, rank, world, tower_precision=args.tower_precision)
        dm.m.load_images(left, right)

        def step(timed=None):
            e = t_tower.start() if timed == "stages" else None
            r = dm.match()
            if e is not None:
                t_tower.stop(e)
            return r
        pairs_per_step, scaling, par = 1, "strong", f"dshard{world}"
    else:
        sgm = what == "tower+cbca+sgm"
        m = StereoMatcher(H, W, D, tower_precision=args.tower_precision, cv_mode=args.cv_mode, sgm=sgm,
                          cbca_iters=CBCA_ITERS if sgm else 0, cbca_L1=CBCA_L1, cbca_tau=CBCA_TAU)
        m.load_images(left, right)
        if what == "cv_wta":
            m.features()
        step = make_step(m, what, t_conv, t_cv, t_tower)
        pairs_per_step, scaling, par = world, "weak", f"pairdp{world}"

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed="conv")
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # per-stage times from a few extra steps outside the timed region (their events would add
    # stream barriers to the timed steps)
    for _ in range(min(args.steps, 5)):
        step(timed="stages")
    torch.cuda.synchronize()
    tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    elapsed = float(tt.item())

    vox = float(H) * W * D
    value = vox * pairs_per_step * args.steps / elapsed / 1e6
    ms_step = elapsed / args.steps * 1e3

    roof = None
    stages = {}
    if what == "tower+cbca+sgm" and (args.mode == "pairdp" or world == 1):
        stages["tower_ms_pair"] = t_tower.mean_ms()
        stages["gpu_path_ms"] = t_cv.mean_ms()
        tim = {}
        m.sgm_path(post=True, timings=tim)           # one synchronised pass, per-stage wall times
        stages.update({f"{k}_ms": v * 1e3 for k, v in tim.items()})
        b = m.sgm_bufs
        # the SGM pair (both sides, 8 directions = 8 launches) timed alone with HIP events
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.sgm_8path_wta_pair(b["cv"][0], b["pen"][0], b["S"][0], b["disp"][0], b["cv"][1], b["pen"][1],
                               b["S"][1], b["disp"][1], zero_du_penalties=True)
        e1.record()
        torch.cuda.synchronize()
        sgm_ms = e0.elapsed_time(e1)
        # per side: UD+DU pass reads C, writes S (8 B/voxel); 5 passes read C, S and write S (12 B);
        # the last pass (WTA fused) reads C, S (8 B) and writes 4 B per pixel
        sgm_bytes = 2 * (76.0 * vox + 4.0 * H * W)
        # one CBCA iteration of both sides (sde_cbca_pair: 2 launches; S buffers as scratch, as in sgm_path)
        e0.record()
        ops.cbca_pair(b["cv"][0], b["cv"][1], b["arms"][0], b["arms"][1], CBCA_L1, 1, tmp_l=b["S"][0],
                      tmp_r=b["S"][1])
        e1.record()
        torch.cuda.synchronize()
        cb_ms = e0.elapsed_time(e1)
        stages["cbca_pair_iter_ms"] = cb_ms
        # 2 sides x 2 passes x (read + write) x 4 B
        stages["cbca_pair_iter_hbm_GBs"] = 2 * 16.0 * vox / (cb_ms * 1e-3) / 1e9
        stages["sgm_pair_ms"] = sgm_ms
        ach = sgm_bytes / (sgm_ms * 1e-3) / 1e9
        roof = {"kernel": "sgm_scan_kernel (8-path SGM + WTA, both sides, 7 launches: DU folded into UD, WTA "
                          "into DU-RL)", "bound": "hbm",
                "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": ach / PEAK_HBM_GBS,
                "traffic": None,
                "per_launch": f"2 sides x (8 + 5 x 12 + 8) B/voxel x {vox / 1e6:.0f} Mvox + disp = "
                              f"{sgm_bytes / 1e9:.2f} GB over {sgm_ms:.3f} ms (7 launches)"}
    elif args.mode == "pairdp" or world == 1:
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
            if m.tower_precision in ("bf16x6", "f16x3"):
                # 6 bf16 / 3 f16 partial products per fp32 product: the roof is the dense bf16/f16 MFMA rate
                k, kt = (6, "bf16") if m.tower_precision == "bf16x6" else (3, "f16")
                ach = k * fl / (conv_ms * 1e-3) / 1e12
                roof = {"kernel": f"conv64_x6p_kernel<false,false,true,true,{str(kt == 'f16').lower()}> "
                                  f"(tower layer 3, {m.tower_precision})", "bound": "mfma",
                        "achieved": ach, "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_BF16_TFLOPS,
                        "traffic": None,
                        "per_launch": f"{k} x {fl / 1e9:.2f} GFLOP {kt} (2 images x 2*{hout}*{wout}*64*576 fp32-equivalent) "
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
            # the reference's boundary hands over host arrays: host u8 pair in -> host float disparity
            # out, PCIe copies and synchronisation included (reported beside `value`, never as it)
            for _ in range(2):
                m.load_images(left, right)
                m.match().cpu()
            t0 = time.perf_counter()
            for _ in range(5):
                m.load_images(left, right)
                m.match().cpu()
            stages["ms_per_pair_host_io"] = (time.perf_counter() - t0) / 5 * 1e3
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
        stages["dshard_step_ms"] = t_tower.mean_ms()

    if roof is not None:
        tb, src = measured_traffic(args.workload)
        roof["traffic"] = tb
        roof["traffic_unit"] = "bytes per launch (HBM, PMC)"
        roof["traffic_source"] = src

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(H, W, D, what)

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
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
