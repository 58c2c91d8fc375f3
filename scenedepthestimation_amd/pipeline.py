"""Device-resident stereo matching: buffers allocated once, every stage a libsde launch.

``StereoMatcher`` is the hot path behind both the drop-in function API
(process_functional.py) and bench.py:

    u8 images (HBM) -> z-norm + zero pad -> MC-CNN tower (x2) -> fused cost
    volume + WTA over [d0, d1)                         (configs 1/2, north star)

and the GPU path of ``disparity_compute_by_gpu`` (process_functional.py:1093-1267):

    features -> [H,W,D] L/R volumes -> penalties -> 8-path SGM (L, R) -> WTA
    -> LR check -> LRC fill -> 5x5 median

All buffers are sized for one (H, W, D) problem and reused across calls, so a
call allocates nothing and can be captured into a HIP graph.
"""
from __future__ import annotations

import numpy as np
import torch

from . import mc_cnn, ops


AMAX_WORDS = 64   # f16x3 bound words per image in the tower workspace (TOWER_AMAX_BYTES / 4)
SPLIT_MAX_PIX = 1 << 24   # split activations: fewer input pixels per plane than this (tower.hip SPLIT_MAX_PIX)
# Placement draws of the four SGM volumes (StereoMatcher._place_sgm_volumes): volumes of [MIN, MAX] voxels are
# placed by up to this many allocate-and-time draws (larger ones would hold three 4-volume sets of > 6 GB each).
SGM_PLACEMENT_TRIALS = 16   # round 6: 8 draws missed the fast mode on some boxes (7 slow draws seen in a row)
SGM_PLACEMENT_MIN_VOXELS = 1 << 26
SGM_PLACEMENT_MAX_VOXELS = 1 << 29


def tower_steps(img_pad, packed, nlayers: int, out, ws, precision: str = "f16x3", nf: int = 64, on_launch=None):
    """sde_tower_forward_batch's launch sequence (mc_cnn_brunch.py:31-48), one layer at a time, as a
    generator: the same launches, bound-word memset and image absmax (each image's activations
    packed at its layer's own size rather than the C path's fixed act_stride), so the features are
    bit-identical to ops.tower_forward_batch.  It yields (stage, words) after the
    image bound (stage 1) and after every layer l < nlayers (stage l): the points at which a caller
    may combine the f16x3 bound words of row bands (all-reduce MAX, parallel.py) before the next
    layer reads them.  on_launch(layer, launch): optional wrapper around each layer's launch (timing).

    img_pad f32 [N, H+2L, W+2L] (contiguous), out f32 [N, H, W, nf], ws uint8 of
    ops.tower_batch_workspace_bytes(H, W, N, nlayers) bytes (or more)."""
    L = nlayers
    N, Hp, Wp = img_pad.shape
    H, W = Hp - 2 * L, Wp - 2 * L
    need = ops.tower_batch_workspace_bytes(H, W, N, L, nf)
    if ws.numel() < need:
        raise ValueError("tower workspace too small")
    h2, w2 = H + 2 * (L - 2), W + 2 * (L - 2)
    # between layers: what sde_tower_forward_batch passes -- split activations on the f16x3 tower when
    # built with them (ops.TOWER_SPLIT_ACT; <= 32 layers, < 2^24 pixels), else c-block-major fp32
    sp = ops.TOWER_SPLIT_ACT and precision == "f16x3" and 2 < L <= ops.SCALE_WORD and h2 * w2 < SPLIT_MAX_PIX
    cbl = not sp and precision in ("bf16x6", "f16x3", "f16x3w", "f16x3m32")
    act = h2 * w2 * nf if L > 2 else 0
    wsf = ws[: 2 * N * act * 4 + N * AMAX_WORDS * 4].view(torch.float32)
    bufs = [wsf[: N * act], wsf[N * act: 2 * N * act]]
    words = wsf[2 * N * act:].view(N, AMAX_WORDS)
    f16 = precision in ("f16x3", "f16x3w", "f16x3m32")
    if f16:
        words.zero_()
        ops.absmax_batch(img_pad, words)
    yield 1, words

    def run(layer, fn):
        if on_launch is None:
            fn()
        else:
            on_launch(layer, fn)

    hin, win = H + 2 * L - 4, W + 2 * L - 4
    first = out if L == 2 else bufs[0][: N * hin * win * nf].view(N, hin, win, nf)
    run(2, lambda: ops.tower_layer_batch(img_pad, packed, L, 2, first, nf=nf, precision=precision,
                                         out_cblock=cbl and L > 2, in_absmax=words[:, 0:1] if f16 else None,
                                         out_absmax=words[:, 1:2] if (f16 and L > 2) else None, out_split=sp))
    cur = 0
    for layer in range(3, L + 1):
        yield layer - 1, words
        src = bufs[cur][: N * hin * win * nf].view(N, hin, win, nf)
        o = out if layer == L else bufs[cur ^ 1][: N * (hin - 2) * (win - 2) * nf].view(N, hin - 2, win - 2, nf)
        run(layer, lambda: ops.tower_layer_batch(src, packed, L, layer, o, nf=nf, precision=precision,
                                                 in_cblock=cbl, out_cblock=cbl and layer < L,
                                                 in_absmax=words[:, layer - 2:layer - 1] if f16 else None,
                                                 out_absmax=words[:, layer - 1:layer] if (f16 and layer < L) else None,
                                                 in_split=sp, out_split=sp and layer < L))
        hin, win = hin - 2, win - 2
        cur ^= 1


def run_tower(img_pad, packed, nlayers, out, ws, precision="f16x3", nf=64, combine=None, on_launch=None):
    """Drive tower_steps to the end; combine(words) is applied at every yield (e.g. an all-reduce)."""
    for _stage, words in tower_steps(img_pad, packed, nlayers, out, ws, precision, nf, on_launch):
        if combine is not None:
            combine(words)
    return out


class StereoMatcher:
    def __init__(self, height: int, width: int, ndisp: int, weights=None, nlayers: int = 5,
                 nf: int = 64, device=None, d_range=None, sgm: bool = False, tower_precision: str = "f16x3",
                 cv_mode: str = "certified", cbca_iters: int = 0, cbca_L1: int = 14, cbca_tau: float = 0.02,
                 emit_split: bool = False, sgm_placement_trials: int = SGM_PLACEMENT_TRIALS):
        self.H, self.W, self.D = int(height), int(width), int(ndisp)
        # cross-based aggregation before SGM (build-defined stage; 0 = the reference's GPU path)
        self.cbca_iters, self.cbca_L1, self.cbca_tau = int(cbca_iters), int(cbca_L1), float(cbca_tau)
        self.nlayers, self.nf = int(nlayers), int(nf)
        self.sgm_placement_trials = int(sgm_placement_trials)
        self.sgm_placement_ms = None     # the SGM pair time of each placement draw (_place_sgm_volumes)
        if tower_precision not in ops.TOWER_PRECISIONS:
            raise ValueError(f"tower_precision must be one of {sorted(ops.TOWER_PRECISIONS)}")
        self.tower_precision = tower_precision
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.d0, self.d1 = (0, self.D) if d_range is None else (int(d_range[0]), int(d_range[1]))
        w = mc_cnn.load_weights(weights, self.nlayers)
        hw, hb = mc_cnn.layer_lists(w, self.nlayers)
        packed = ops.pack_tower_weights(hw, hb)
        dev = self.device
        H, W, L = self.H, self.W, self.nlayers
        self.packed = torch.from_numpy(packed).to(dev)
        self.img_u82 = torch.empty((2, H, W), dtype=torch.uint8, device=dev)
        self.img_u8 = [self.img_u82[0], self.img_u82[1]]
        # both images in one allocation: the tower runs the pair per launch (sde_tower_forward_batch)
        self.img_pad2 = torch.empty((2, H + 2 * L, W + 2 * L), dtype=torch.float32, device=dev)
        self.img_pad = [self.img_pad2[0], self.img_pad2[1]]
        n = ops.preprocess_scratch_bytes(H, W)
        self.stats2 = torch.empty((2 * n,), dtype=torch.uint8, device=dev)
        self.stats = [self.stats2[:n], self.stats2[n:]]
        self.feat2 = torch.empty((2, H, W, nf), dtype=torch.float32, device=dev)
        self.feat = [self.feat2[0], self.feat2[1]]
        self._ws = None        # the tower workspace, allocated on first use (see ws)
        self.disp = torch.empty((H, W), dtype=torch.float32, device=dev)
        self.min_cost = torch.empty((H, W), dtype=torch.float32, device=dev)
        self.argmin = torch.empty((H, W), dtype=torch.int32, device=dev)
        self.cv_mode = cv_mode
        self.cv_ws = torch.empty(ops.cv_wta_workspace_bytes(H, W), dtype=torch.uint8, device=dev)
        # optional: bf16 split planes + norm bounds emitted by the tower's last layer, consumed by
        # sde_cv_wta_split.  The default certified path (sde_cv_wta, row-sweep kernel) splits the fp32
        # features itself and reads nothing else, so the planes are not written by default.
        self.split = [ops.new_split(H, W, dev) for _ in range(2)] \
            if (emit_split and cv_mode == "certified" and nlayers >= 2) else None
        self.split_valid = False
        self.sgm_bufs = None
        if sgm:
            self._alloc_sgm()

    @property
    def ws(self):
        """Tower workspace (both images' activations + bound words, ~4 x H x W x 64 floats), allocated
        on first use: a matcher whose tower runs elsewhere (parallel.DisparityShardedMatcher's band
        tower) never holds it."""
        if self._ws is None:
            nws = ops.tower_batch_workspace_bytes(self.H, self.W, 2, self.nlayers, self.nf)
            self._ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=self.device)
        return self._ws

    # -- stages ----------------------------------------------------------------
    def load_images(self, left_u8, right_u8):
        """Host u8 [H,W] arrays (or device tensors) -> resident device images."""
        for dst, src in zip(self.img_u8, (left_u8, right_u8)):
            t = src if isinstance(src, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(src, np.uint8))
            dst.copy_(t, non_blocking=False)

    def features(self, on_launch=None):
        """Preprocess + tower for both images (compute_feature, process_functional.py:11-45).
        on_launch(layer, launch): run the tower layer by layer from Python (tower_steps: the same
        launches, bits and workspace as the one-call path) with each launch wrapped, e.g. timed."""
        ops.preprocess_u8_batch(self.img_u82, self.nlayers, out=self.img_pad2, stats=self.stats2)
        return self.features_from_padded(on_launch)

    def features_from_padded(self, on_launch=None):
        """Tower only, on already-normalised padded images in self.img_pad (the pair per launch)."""
        if on_launch is not None and self.split:
            raise ValueError("on_launch needs the layer-by-layer tower, which does not emit split planes "
                             "(emit_split=True): time the one-call tower instead")
        if on_launch is not None:
            run_tower(self.img_pad2, self.packed, self.nlayers, self.feat2, self.ws, self.tower_precision, self.nf,
                      on_launch=on_launch)
            self.split_valid = False
            return self.feat[0], self.feat[1]
        if self.split:
            for i in range(2):
                ops.tower_forward(self.img_pad[i], self.packed, self.nlayers, self.nf, out=self.feat[i],
                                  workspace=self.ws, precision=self.tower_precision, split=self.split[i])
        else:
            ops.tower_forward_batch(self.img_pad2, self.packed, self.nlayers, self.nf, out=self.feat2,
                                    workspace=self.ws, precision=self.tower_precision)
        self.split_valid = self.split is not None
        return self.feat[0], self.feat[1]

    def cost_wta(self, want=("disp",)):
        """Fused cost volume + WTA over this matcher's disparity range [d0, d1).  In certified mode with
        emit_split=True the tower-emitted split planes are used (sde_cv_wta_split) when the current
        features came from this matcher's tower; otherwise sde_cv_wta reads the fp32 features."""
        if self.cv_mode == "certified" and self.split_valid:
            return ops.cv_wta_split(self.feat[0], self.feat[1], self.split[0], self.split[1], self.d0, self.d1,
                                    disp=self.disp if "disp" in want else None,
                                    min_cost=self.min_cost if "min" in want else None,
                                    argmin=self.argmin if "argmin" in want else None, want=(),
                                    workspace=self.cv_ws)
        return ops.cv_wta(self.feat[0], self.feat[1], self.d0, self.d1,
                          disp=self.disp if "disp" in want else None,
                          min_cost=self.min_cost if "min" in want else None,
                          argmin=self.argmin if "argmin" in want else None, want=(),
                          mode=self.cv_mode, workspace=self.cv_ws)

    def match(self):
        """One pass of the hot path on the resident images: features + fused CV/WTA -> disparity."""
        self.features()
        self.cost_wta()
        return self.disp

    # -- GPU path of disparity_compute_by_gpu ---------------------------------
    def _place_sgm_volumes(self, pen, disp):
        """The four [H,W,D] volumes of the GPU path (cost L/R, SGM S L/R), placed by allocate-and-time draws.

        The 7-launch SGM pair moves the same bytes through any four volumes, yet on MI355X it runs in one of two
        modes by where the allocation lands in HBM: ~5.3 or ~5.7-5.8 ms at 1024^2 x 192 (LR/RL 0.81 vs 0.95 ms
        per launch, the diagonals 0.80 vs 0.85; the same virtual addresses can come back in either mode,
        row strides and offsets inside one allocation do not decide it, the box's thermal / power state does not
        either -- tools/sgm_*_probe.py).  So for large volumes each draw allocates a fresh
        set (the previous one still held, so the draw gets other memory), times one pair on zero costs, and the
        fastest set is kept; the draws stop once one beats the slowest seen by 6 % (both modes seen).  One-time
        cost: ~20 ms per draw."""
        H, W, D, dev = self.H, self.W, self.D, self.device

        def new_set():
            return [torch.empty((H, W, D), dtype=torch.float32, device=dev) for _ in range(4)]
        trials = self.sgm_placement_trials if SGM_PLACEMENT_MIN_VOXELS <= H * W * D <= SGM_PLACEMENT_MAX_VOXELS else 1
        if trials <= 1:
            return new_set()
        for p in pen:
            p.zero_()

        def pair_ms(v):
            for t in v:
                t.zero_()
            run = lambda: ops.sgm_8path_wta_pair(v[0], pen[0], v[2], disp[0], v[1], pen[1], v[3], disp[1],  # noqa: E731
                                                 zero_du_penalties=True)
            run()
            best = float("inf")
            for _ in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run()
                e1.record()
                torch.cuda.synchronize(dev)
                best = min(best, e0.elapsed_time(e1))
            return best
        best, best_ms, worst, prev, times = None, float("inf"), 0.0, None, []
        for _ in range(trials):
            cur = new_set()
            ms = pair_ms(cur)
            times.append(ms)
            worst = max(worst, ms)
            if ms < best_ms:
                best, best_ms = cur, ms
            prev = cur
            torch.cuda.empty_cache()
            if best_ms <= 0.94 * worst:
                break
        del prev, cur
        torch.cuda.empty_cache()
        self.sgm_placement_ms = times
        return best

    def _alloc_sgm(self):
        H, W, D, dev = self.H, self.W, self.D, self.device
        pen = [torch.empty((H, W, 16), dtype=torch.float32, device=dev) for _ in range(2)]
        disp = [torch.empty((H, W), dtype=torch.float32, device=dev) for _ in range(2)]
        cvl, cvr, sl, sr = self._place_sgm_volumes(pen, disp)
        # the right volume starts as the GPU path's invalid fill (1.0): with aggregation on, the cost
        # volume sweep writes the left volume only and sde_cbca_lr the right one's valid voxels, so its
        # invalid voxels (x + d >= W) keep this fill -- the value the two-volume sweep writes there
        cvr.fill_(1.0)
        self.sgm_bufs = dict(
            cv=[cvl, cvr],
            pen=pen,
            S=[sl, sr],
            disp=disp,
            lrc=[torch.empty((H, W), dtype=torch.uint8, device=dev) for _ in range(2)],
            disp_a=torch.empty((H, W), dtype=torch.float32, device=dev),
            disp_b=torch.empty((H, W), dtype=torch.float32, device=dev),
        )
        if self.cbca_iters > 0:
            self.sgm_bufs["arms"] = [torch.empty((H, W), dtype=torch.int32, device=dev) for _ in range(2)]
            self.sgm_bufs["cbca_ws"] = torch.empty((ops.cbca_workspace_bytes(H, W),), dtype=torch.uint8, device=dev)

    def cbca(self, cv_l, cv_r, img_l, img_r):
        """Cross-based aggregation (build-defined) of the left [H,W,D] volume in
        place, and the right volume derived from it.  Arms come from the z-normalised images (the
        tower's input normalisation).

        cv_r is an OUTPUT: its valid voxels (x + d < W) are overwritten with the shear of the aggregated
        cv_l and their input is never read -- correct only because the GPU path's right volume IS the
        left one's shear (one sweep computes each voxel once, sec. 3.1).  Its invalid voxels are kept.
        For two independent volumes use ops.cbca_pair."""
        if self.sgm_bufs is None or "arms" not in self.sgm_bufs:
            saved, self.cbca_iters = self.cbca_iters, max(self.cbca_iters, 1)
            self._alloc_sgm()
            self.cbca_iters = saved
        b, P, H, W = self.sgm_bufs, self.nlayers, self.H, self.W
        for k, img in enumerate((img_l, img_r)):
            ops.preprocess_u8(img, P, out=self.img_pad[k], stats=self.stats[k])
            ops.cbca_arms(self.img_pad[k][P:P + H, P:P + W], self.cbca_L1, self.cbca_tau, out=b["arms"][k])
        # the right volume is the left one's shear (valid voxels), so its aggregation is the shear of the
        # left one's (definition v2): one volume aggregated, then one shear pass writes cv_r's valid voxels
        # (their input is not read; its invalid voxels are kept).  The SGM S buffer (written later,
        # overwrite mode) is the scratch.
        ops.cbca_lr(cv_l, cv_r, b["arms"][0], b["arms"][1], self.cbca_L1, self.cbca_iters, tmp=b["S"][0],
                    workspace=b["cbca_ws"])
        return cv_l, cv_r

    def sgm_path(self, fl=None, fr=None, img_l=None, img_r=None, timings=None, post=True):
        """process_functional.py:1093-1267 on device tensors; returns (disp_l, disp_r).

        timings: optional dict receiving per-stage seconds (synchronised)."""
        import time
        if self.sgm_bufs is None:
            self._alloc_sgm()
        b = self.sgm_bufs
        fl = self.feat[0] if fl is None else fl
        fr = self.feat[1] if fr is None else fr
        img_l = self.img_u8[0] if img_l is None else img_l
        img_r = self.img_u8[1] if img_r is None else img_r

        def mark(name, t0):
            if timings is not None:
                torch.cuda.synchronize(self.device)
                t1 = time.time()
                timings[name] = timings.get(name, 0.0) + (t1 - t0)
                return t1
            return t0

        t = time.time() if timings is not None else 0.0
        # process_functional.py:120-131.  With aggregation the right volume comes from sde_cbca_lr (the
        # aggregated left volume's shear), so the sweep writes the left one only.
        ops.cost_volume(fl, fr, self.D, layout="HWD", right=self.cbca_iters <= 0, invalid=1.0,
                        out_left=b["cv"][0], out_right=b["cv"][1] if self.cbca_iters <= 0 else None)
        t = mark("cost_volume", t)
        if self.cbca_iters > 0:
            self.cbca(b["cv"][0], b["cv"][1], img_l, img_r)
            t = mark("cbca", t)
        ops.sgm_penalties(img_l, out=b["pen"][0])
        ops.sgm_penalties(img_r, out=b["pen"][1])
        # both sides per launch (the reference's k loop); S := 8-path sum, no zero-fill pass
        # penalties from sgm_penalties (channels 0/1 zero), finite costs: DU folds into UD;
        # WTA_and_SupixelRefinement_kernel (:800-837) fused into the last direction
        ops.sgm_8path_wta_pair(b["cv"][0], b["pen"][0], b["S"][0], b["disp"][0], b["cv"][1], b["pen"][1],
                               b["S"][1], b["disp"][1], zero_du_penalties=True)
        t = mark("sgm", t)
        if not post:
            return b["disp"][0], b["disp"][1]
        b["lrc"][0].zero_()
        b["lrc"][1].zero_()
        ops.lr_check(b["disp"][0], b["disp"][1], b["lrc"][0], b["lrc"][1])
        ops.lrc_fill(b["disp"][0], b["lrc"][0], out=b["disp_a"])
        t = mark("lrc", t)
        # Median_Filter_kernel(d_disparityl_a, d_disparityr_a, d_disparityl, d_disparityr) (:1250):
        # the interior of disp_l becomes the median of the LRC-filled map.  The reference's
        # right input d_disparityr_a is never written (:1227); here the right map is filtered
        # from its own WTA output (documented divergence, parity unpinned).
        disp_r_src = b["disp_b"]
        disp_r_src.copy_(b["disp"][1])
        ops.median5(b["disp_a"], b["disp"][0])
        ops.median5(disp_r_src, b["disp"][1])
        mark("filter", t)
        return b["disp"][0], b["disp"][1]
