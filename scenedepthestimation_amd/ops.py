"""Tensor-level wrappers over the C ABI (include/sde.h).

Every op takes CUDA (HIP) torch tensors, checks dtype / contiguity / shape on
the host, launches on torch's current stream and returns torch tensors.  torch
is only plumbing here (device memory, streams); all arithmetic runs in the HIP
kernels of libsde.so.  There is no CPU fallback: on a machine without a GPU
these functions raise.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import (SDE_LAYOUT_DHW, SDE_LAYOUT_HWD, SDE_SIDE_LEFT, SDE_SIDE_RIGHT, SDE_WTA_INIT_D0,
                   SDE_WTA_INIT_INF, check, lib)

LAYOUTS = {"DHW": SDE_LAYOUT_DHW, "HWD": SDE_LAYOUT_HWD}
RULES = {"inf": SDE_WTA_INIT_INF, "d0": SDE_WTA_INIT_D0}


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _need(t: torch.Tensor, name: str, dtype=torch.float32, shape=None):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"{name} must live on the GPU (got {t.device}); libsde has no CPU path")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if shape is not None and tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)} (got {tuple(t.shape)})")
    return t.data_ptr()


def _empty(shape, dtype, like):
    return torch.empty(shape, dtype=dtype, device=like.device)


def _feat_pair(fl, fr):
    if fl.dim() != 3 or tuple(fl.shape) != tuple(fr.shape):
        raise ValueError(f"features must be matching [H,W,C] tensors, got {tuple(fl.shape)} / {tuple(fr.shape)}")
    H, W, C = fl.shape
    return _need(fl, "featuresl", shape=(H, W, C)), _need(fr, "featuresr", shape=(H, W, C)), H, W, C


# ----------------------------------------------------------------------------
# cost volume / WTA (process_functional.py:48-131, 800-837)
# ----------------------------------------------------------------------------
def cost_volume(fl, fr, ndisp: int, layout: str = "DHW", right: bool = False, invalid=None,
                out_left=None, out_right=None, left: bool = True):
    """Exact cost volume.  DHW: compute_cost_volume (invalid -0.0).  HWD: GPU-path layout
    with left and optionally right volumes (invalid 1.0, process_functional.py:1111); both
    sides come from one pass (each voxel computed once, stored twice)."""
    pl, pr, H, W, C = _feat_pair(fl, fr)
    lay = LAYOUTS[layout]
    if invalid is None:
        invalid = -0.0 if layout == "DHW" else 1.0
    shape = (ndisp, H, W) if layout == "DHW" else (H, W, ndisp)
    if not left and not right:
        raise ValueError("nothing to compute")
    ol = orr = None
    sides = 0
    if left:
        if out_left is None:
            out_left = _empty(shape, torch.float32, fl)
        ol = _need(out_left, "out_left", shape=shape)
        sides |= SDE_SIDE_LEFT
    if right:
        if layout != "HWD":
            raise ValueError("the right volume exists in the HWD (GPU-path) layout only")
        if out_right is None:
            out_right = _empty(shape, torch.float32, fl)
        orr = _need(out_right, "out_right", shape=shape)
        sides |= SDE_SIDE_RIGHT
    check(lib.sde_cost_volume(pl, pr, H, W, C, int(ndisp), lay, sides, ctypes.c_float(invalid), ol, orr,
                              _stream()), "sde_cost_volume")
    if not left:
        return out_right
    return (out_left, out_right) if right else out_left


CV_MODES = {"exact": _lib.SDE_CV_EXACT, "certified": _lib.SDE_CV_CERTIFIED}


def cv_wta_workspace_bytes(H: int, W: int) -> int:
    return int(lib.sde_cv_wta_workspace_bytes(H, W))


def cv_wta(fl, fr, d0: int, d1: int, disp=None, min_cost=None, argmin=None, want=("disp",), mode: str = "certified",
           workspace=None):
    """Fused cost volume + first-min over [d0, d1): WTA1(compute_cost_volume(fl, fr, d1)) when d0 = 0.

    mode 'exact' (VALU, NumPy order for every voxel) or 'certified' (bf16x3 MFMA scores + error bound,
    exact resolution of uncertified pixels): identical outputs.  workspace: uint8 tensor of
    cv_wta_workspace_bytes(H, W) bytes (allocated if None); its first int32 holds the number of
    pixels resolved exactly after the call."""
    pl, pr, H, W, C = _feat_pair(fl, fr)
    if "disp" in want and disp is None:
        disp = _empty((H, W), torch.float32, fl)
    if "min" in want and min_cost is None:
        min_cost = _empty((H, W), torch.float32, fl)
    if "argmin" in want and argmin is None:
        argmin = _empty((H, W), torch.int32, fl)
    pd = _need(disp, "disp", shape=(H, W)) if disp is not None else None
    pm = _need(min_cost, "min_cost", shape=(H, W)) if min_cost is not None else None
    pa = _need(argmin, "argmin", dtype=torch.int32, shape=(H, W)) if argmin is not None else None
    md = CV_MODES[mode]
    pws, wsb = None, 0
    if md == _lib.SDE_CV_CERTIFIED:
        need = cv_wta_workspace_bytes(H, W)
        if workspace is None:
            workspace = torch.empty(need, dtype=torch.uint8, device=fl.device)
        pws, wsb = _need(workspace, "workspace", dtype=torch.uint8), workspace.numel()
    check(lib.sde_cv_wta(pl, pr, H, W, C, int(d0), int(d1), pd, pm, pa, md, pws, wsb, _stream()), "sde_cv_wta")
    return disp, min_cost, argmin


def cv_wta_split_workspace_bytes(H: int, W: int) -> int:
    return int(lib.sde_cv_wta_split_workspace_bytes(H, W))


def cv_wta_split(fl, fr, split_l, split_r, d0: int, d1: int, disp=None, min_cost=None, argmin=None,
                 workspace=None, want=("disp",)):
    """Certified fused CV + WTA on pre-split operands (tower-emitted or feature_split)."""
    pl, pr, H, W, C = _feat_pair(fl, fr)
    if "disp" in want and disp is None:
        disp = _empty((H, W), torch.float32, fl)
    if "min" in want and min_cost is None:
        min_cost = _empty((H, W), torch.float32, fl)
    if "argmin" in want and argmin is None:
        argmin = _empty((H, W), torch.int32, fl)
    pd = _need(disp, "disp", shape=(H, W)) if disp is not None else None
    pm = _need(min_cost, "min_cost", shape=(H, W)) if min_cost is not None else None
    pa = _need(argmin, "argmin", dtype=torch.int32, shape=(H, W)) if argmin is not None else None
    if workspace is None:
        workspace = torch.empty(cv_wta_split_workspace_bytes(H, W), dtype=torch.uint8, device=fl.device)
    lh, ll, ln = _split_ptrs(split_l, (H, W))
    rh, rl, rn = _split_ptrs(split_r, (H, W))
    check(lib.sde_cv_wta_split(pl, pr, lh, ll, ln, rh, rl, rn, H, W, int(d0), int(d1), pd, pm, pa,
                               _need(workspace, "workspace", dtype=torch.uint8), workspace.numel(), _stream()),
          "sde_cv_wta_split")
    return disp, min_cost, argmin


def cv_wta_fixups(workspace) -> int:
    """Number of pixels the last certified cv_wta call resolved with the exact scan (synchronises): the sum of
    the workspace's 64 counter words (one per 256-disparity chunk on the chunked path, word 0 otherwise)."""
    return int(workspace[:256].view(torch.int32).sum().item())


def wta(vol, layout: str = "DHW", rule: str = "inf", out=None):
    """First-min over d: WTA1 (DHW), WTA (HWD) or the SGM WTA kernel (HWD, rule='d0')."""
    if vol.dim() != 3:
        raise ValueError("volume must be 3-D")
    if layout == "DHW":
        D, H, W = vol.shape
    else:
        H, W, D = vol.shape
    pv = _need(vol, "volume")
    if out is None:
        out = _empty((H, W), torch.float32, vol)
    po = _need(out, "disp", shape=(H, W))
    check(lib.sde_wta(pv, H, W, D, LAYOUTS[layout], RULES[rule], po, _stream()), "sde_wta")
    return out


def argmin_merge(mins, args, out=None):
    """Ordered merge of per-shard (min [S,H,W], argmin [S,H,W]) -> float32 disparity [H,W]."""
    S = mins.shape[0]
    pm = _need(mins, "mins")
    pa = _need(args, "args", dtype=torch.int32, shape=tuple(mins.shape))
    npix = int(np.prod(mins.shape[1:]))
    if out is None:
        out = _empty(tuple(mins.shape[1:]), torch.float32, mins)
    po = _need(out, "disp")
    check(lib.sde_argmin_merge(pm, pa, S, npix, po, _stream()), "sde_argmin_merge")
    return out


# ----------------------------------------------------------------------------
# MC-CNN tower (mc_cnn_brunch.py:31-48) and preprocessing (match_single.py:34-43)
# ----------------------------------------------------------------------------
def tower_packed_floats(nlayers: int, nf: int = 64) -> int:
    n = lib.sde_tower_packed_floats(nlayers, nf)
    if n < 0:
        raise ValueError(f"unsupported tower shape nlayers={nlayers} nf={nf}")
    return int(n)


def pack_tower_weights(hwio_list, bias_list) -> np.ndarray:
    """Pack HWIO weights / biases (host numpy) into the device blob layout (host-side C helper)."""
    L = len(hwio_list)
    nf = int(hwio_list[0].shape[-1])
    ws = [np.ascontiguousarray(w, dtype=np.float32) for w in hwio_list]
    bs = [np.ascontiguousarray(b, dtype=np.float32) for b in bias_list]
    for l, (w, b) in enumerate(zip(ws, bs)):
        cin = 1 if l == 0 else nf
        if w.shape != (3, 3, cin, nf) or b.shape != (nf,):
            raise ValueError(f"layer {l + 1}: expected weights (3,3,{cin},{nf}) and biases ({nf},), "
                             f"got {w.shape} / {b.shape}")
    out = np.empty(tower_packed_floats(L, nf), np.float32)
    wp = (ctypes.c_void_p * L)(*[w.ctypes.data for w in ws])
    bp = (ctypes.c_void_p * L)(*[b.ctypes.data for b in bs])
    check(lib.sde_tower_pack_weights(wp, bp, L, nf, out.ctypes.data), "sde_tower_pack_weights")
    return out


def tower_workspace_bytes(H: int, W: int, nlayers: int, nf: int = 64) -> int:
    return int(lib.sde_tower_workspace_bytes(H, W, nlayers, nf))


# "f16x3w": f16x3 with the Winograd F(2x2, 3x3) kernel for layers 3..L (SDE_TOWER_WINOGRAD)
# "f16x3m32": f16x3 with layers 3..L on the 32x32x16 direct kernel (SDE_TOWER_MFMA32; the default f16x3
# runs them on the 16x16x32 kernel)
TOWER_PRECISIONS = {"fp32": _lib.SDE_TOWER_FP32, "bf16x6": _lib.SDE_TOWER_BF16X6, "f16x3": _lib.SDE_TOWER_F16X3,
                    "f16x3w": _lib.SDE_TOWER_F16X3 | _lib.SDE_TOWER_WINOGRAD,
                    "f16x3m32": _lib.SDE_TOWER_F16X3 | _lib.SDE_TOWER_MFMA32}


def _split_ptrs(split, shape):
    """split = (hi int16 [..., 64], lo int16 [..., 64], norm f32 [...]) or None -> three pointers."""
    if split is None:
        return None, None, None
    hi, lo, nrm = split
    return (_need(hi, "feat_hi", dtype=torch.int16, shape=shape + (64,)),
            _need(lo, "feat_lo", dtype=torch.int16, shape=shape + (64,)),
            _need(nrm, "feat_norm", shape=shape))


def new_split(H: int, W: int, device):
    """Buffers for bf16 split planes + norm bound of an [H,W,64] feature map."""
    return (torch.empty((H, W, 64), dtype=torch.int16, device=device),
            torch.empty((H, W, 64), dtype=torch.int16, device=device),
            torch.empty((H, W), dtype=torch.float32, device=device))


def feature_split(feat, split=None):
    """[H,W,64] f32 -> (hi, lo, norm) for the certified cost volume (sde_feature_split)."""
    H, W, C = feat.shape
    if split is None:
        split = new_split(H, W, feat.device)
    ph, pl, pn = _split_ptrs(split, (H, W))
    check(lib.sde_feature_split(_need(feat, "features"), H * W, C, ph, pl, pn, _stream()), "sde_feature_split")
    return split


def tower_forward(img_pad, packed, nlayers: int, nf: int = 64, out=None, workspace=None, precision: str = "fp32",
                  split=None):
    """img_pad: f32 [H+2L, W+2L] -> L2-normalised features f32 [H, W, nf].
    precision: 'fp32' (fp32 MFMA), 'bf16x6' (exact 3-way bf16 split, 6 partial products, fp32 accumulate) or
    'f16x3' (power-of-two scaled exact 2-way fp16 split, 3 partial products, fp32 accumulate).
    split: optional (hi, lo, norm) buffers the last layer's epilogue fills (certified cost volume input)."""
    Hp, Wp = img_pad.shape
    H, W = Hp - 2 * nlayers, Wp - 2 * nlayers
    if H <= 0 or W <= 0:
        raise ValueError("padded image smaller than the tower's receptive field")
    pi = _need(img_pad, "img_pad")
    pw = _need(packed, "packed weights", shape=(tower_packed_floats(nlayers, nf),))
    if out is None:
        out = _empty((H, W, nf), torch.float32, img_pad)
    po = _need(out, "features", shape=(H, W, nf))
    need = tower_workspace_bytes(H, W, nlayers, nf)
    if need > 0 and workspace is None:
        workspace = torch.empty(need, dtype=torch.uint8, device=img_pad.device)
    pws = _need(workspace, "workspace", dtype=torch.uint8) if need > 0 else None
    wsb = workspace.numel() if need > 0 else 0
    ph, pl_, pn = _split_ptrs(split, (H, W))
    check(lib.sde_tower_forward(pi, H, W, pw, nlayers, nf, po, pws, wsb, TOWER_PRECISIONS[precision], ph, pl_, pn,
                                _stream()), "sde_tower_forward")
    return out


def absmax(x, out):
    """out (f32 [1] device) = max(out, max |x|) (sde_absmax_f32)."""
    check(lib.sde_absmax_f32(_need(x, "absmax input"), x.numel(), _need(out, "absmax word", shape=(1,)), _stream()),
          "sde_absmax_f32")
    return out


def set_persistent_grid(cus: int = 0):
    """Cap the persistent tower kernels' grid at `cus` workgroups (0: one per device CU), for a tower that
    shares the device with work on CU-masked streams (sde_set_persistent_grid)."""
    check(lib.sde_set_persistent_grid(int(cus)), "sde_set_persistent_grid")


def tower_batch_workspace_bytes(H: int, W: int, nimg: int, nlayers: int, nf: int = 64) -> int:
    return int(lib.sde_tower_batch_workspace_bytes(H, W, nimg, nlayers, nf))


def tower_forward_batch(img_pad, packed, nlayers: int, nf: int = 64, out=None, workspace=None,
                        precision: str = "f16x3"):
    """img_pad: f32 [N, H+2L, W+2L] -> features f32 [N, H, W, nf], all N images per launch
    (sde_tower_forward_batch); each image's result equals tower_forward on it alone."""
    N, Hp, Wp = img_pad.shape
    H, W = Hp - 2 * nlayers, Wp - 2 * nlayers
    if H <= 0 or W <= 0:
        raise ValueError("padded image smaller than the tower's receptive field")
    pi = _need(img_pad, "img_pad")
    pw = _need(packed, "packed weights", shape=(tower_packed_floats(nlayers, nf),))
    if out is None:
        out = _empty((N, H, W, nf), torch.float32, img_pad)
    po = _need(out, "features", shape=(N, H, W, nf))
    need = tower_batch_workspace_bytes(H, W, N, nlayers, nf)
    if need > 0 and workspace is None:
        workspace = torch.empty(need, dtype=torch.uint8, device=img_pad.device)
    pws = _need(workspace, "workspace", dtype=torch.uint8) if need > 0 else None
    wsb = workspace.numel() if need > 0 else 0
    check(lib.sde_tower_forward_batch(pi, N, H, W, pw, nlayers, nf, po, pws, wsb, TOWER_PRECISIONS[precision],
                                      None, None, None, _stream()), "sde_tower_forward_batch")
    return out


def absmax_batch(x, out):
    """out [N, k] (f32 device, column 0 used) = max(out, max |x[i]|) per image i of x [N, ...]
    (sde_absmax_f32_batch, one launch)."""
    N = x.shape[0]
    _need(x, "absmax input")
    if out.dtype != torch.float32 or not out.is_cuda or out.shape[0] != N or out.stride(1) != 1:
        raise ValueError("absmax words must be a float32 [N, k] device tensor with unit column stride")
    check(lib.sde_absmax_f32_batch(x.data_ptr(), N, x[0].numel(), out.data_ptr(), out.stride(0), _stream()),
          "sde_absmax_f32_batch")
    return out


SCALE_WORD = 32   # split activations: 2^sigma at bound word + 32 (sde.h SDE_TOWER_OUT_SPLIT)
AMAX_ROW_WORDS = 64   # a batch's bound-word row per image (tower.hip TOWER_AMAX_BYTES / 4)
# whether sde_tower_forward* pass split activations between the default f16x3 tower's 64->64 layers, as built
# (sde_tower_split_act(), tower.hip SDE_SPLIT_ACT; the layer-by-layer drivers in pipeline.py follow it to stay
# bit-identical)
TOWER_SPLIT_ACT = bool(lib.sde_tower_split_act())


def _layout_flags(flags, in_cblock, out_cblock, in_split, out_split):
    if in_cblock:
        flags |= _lib.SDE_TOWER_IN_CBLOCK
    if out_cblock:
        flags |= _lib.SDE_TOWER_OUT_CBLOCK
    if in_split:
        flags |= _lib.SDE_TOWER_IN_SPLIT
    if out_split:
        flags |= _lib.SDE_TOWER_OUT_SPLIT
    return flags


def _check_scale_word(words, rows, name):
    """Split activations read / write words[i * stride + 32]: the storage behind the word view must hold it."""
    if words is None:
        return
    stride = words.stride(0) if words.dim() > 1 else 0
    last = words.storage_offset() + (rows - 1) * stride + SCALE_WORD
    if words.untyped_storage().nbytes() < (last + 1) * 4:
        raise ValueError(f"{name}: split activations need the bound-word array to extend {SCALE_WORD} words "
                         "past each image's word (the scale word)")


def tower_layer(inp, packed, nlayers: int, layer: int, out, nf: int = 64, precision: str = "fp32", split=None,
                in_cblock: bool = False, out_cblock: bool = False, in_absmax=None, out_absmax=None,
                in_split: bool = False, out_split: bool = False):
    """One tower layer = one kernel launch (layer 2 = conv1+conv2 fused from the padded image).
    in_cblock / out_cblock (bf16x6, f16x3): intermediate activations in the c-block-major layout
    [nf/16][h][w][16] that tower_forward uses between layers (tensors keep their [h, w, nf]
    shape; only the element order differs).
    in_split / out_split (f16x3): the split-activation layout the default f16x3 tower_forward uses between
    layers (16 planes [cblk32][part][quarter] of [h][w][8 fp16], same bytes as [h, w, nf] f32); the scale
    2^sigma travels at in_absmax / out_absmax + 32 (views into a >= 33-word array).
    in_absmax / out_absmax (f16x3): f32 [1] device words -- a bound of |input| (|image| for layer
    2) and the word this layer maxes its outputs into (zeroed by the caller)."""
    flags = _layout_flags(TOWER_PRECISIONS[precision], in_cblock, out_cblock, in_split, out_split)
    if in_split:
        _check_scale_word(in_absmax, 1, "in_absmax")
    if out_split:
        _check_scale_word(out_absmax, 1, "out_absmax")
    if layer == 2:
        Hin, Win = inp.shape
        oshape = (Hin - 4, Win - 4, nf)
    else:
        Hin, Win, _ = inp.shape
        oshape = (Hin - 2, Win - 2, nf)
    pin = _need(in_absmax, "in_absmax", shape=(1,)) if in_absmax is not None else None
    pout = _need(out_absmax, "out_absmax", shape=(1,)) if out_absmax is not None else None
    check(lib.sde_tower_layer_scaled(_need(inp, "layer input"), Hin, Win,
                                     _need(packed, "packed weights", shape=(tower_packed_floats(nlayers, nf),)),
                                     nlayers, nf, layer, _need(out, "layer output", shape=oshape),
                                     flags, *_split_ptrs(split, oshape[:2]), pin, pout, _stream()),
          "sde_tower_layer_scaled")
    return out


def tower_layer_batch(inp, packed, nlayers: int, layer: int, out, nf: int = 64, precision: str = "f16x3",
                      in_cblock: bool = False, out_cblock: bool = False, in_absmax=None, out_absmax=None,
                      in_split: bool = False, out_split: bool = False):
    """tower_layer over a batch per launch: inp [N, Hin, Win] (layer 2) or [N, Hin, Win, nf], out
    [N, h, w, nf]; in_absmax / out_absmax (f16x3): [N, k] device words, column 0 used (row stride k;
    k > 32 with split activations, whose scale word is column 32)."""
    flags = _layout_flags(TOWER_PRECISIONS[precision], in_cblock, out_cblock, in_split, out_split)
    N, Hin, Win = inp.shape[:3]
    if in_split:
        _check_scale_word(in_absmax, N, "in_absmax")
    if out_split:
        _check_scale_word(out_absmax, N, "out_absmax")
    if (in_split or out_split) and N > 1:
        for words, name in ((in_absmax, "in_absmax"), (out_absmax, "out_absmax")):
            if words is not None and words.stride(0) < AMAX_ROW_WORDS:
                raise ValueError(f"{name}: split activations over a batch need rows of >= {AMAX_ROW_WORDS} bound words "
                                 f"(got a row stride of {words.stride(0)}): a layer's scale word is {SCALE_WORD} "
                                 "words past its bound word")
    sh = 4 if layer == 2 else 2
    oshape = (N, Hin - sh, Win - sh, nf)
    ws = 0
    pin = pout = None
    if in_absmax is not None:
        pin, ws = in_absmax.data_ptr(), in_absmax.stride(0)
    if out_absmax is not None:
        pout = out_absmax.data_ptr()
    _need(inp, "layer input")
    _need(out, "layer output", shape=oshape)
    check(lib.sde_tower_layer_batch(inp.data_ptr(), N, inp[0].numel(), Hin, Win,
                                    _need(packed, "packed weights", shape=(tower_packed_floats(nlayers, nf),)),
                                    nlayers, nf, layer, out.data_ptr(), out[0].numel(), flags, pin, pout, ws,
                                    _stream()), "sde_tower_layer_batch")
    return out


def preprocess_scratch_bytes(H: int, W: int) -> int:
    """Device scratch one image's preprocess needs (sde_preprocess_scratch_bytes)."""
    n = int(lib.sde_preprocess_scratch_bytes(int(H), int(W)))
    if n < 0:
        raise ValueError("invalid image shape")
    return n


def preprocess_u8(img_u8, pad: int, out=None, stats=None):
    """u8 [H,W] -> zero-padded z-normalised f32 [H+2p, W+2p] on the device, bit-identical to
    NumPy's (I - np.mean(I)) / np.std(I) on the float32 image (match_single.py:40-41).
    stats: optional uint8 scratch tensor of preprocess_scratch_bytes(H, W) bytes."""
    H, W = img_u8.shape
    pi = _need(img_u8, "image", dtype=torch.uint8)
    nb = preprocess_scratch_bytes(H, W)
    if out is None:
        out = _empty((H + 2 * pad, W + 2 * pad), torch.float32, img_u8)
    if stats is None:
        stats = _empty((nb,), torch.uint8, img_u8)
    check(lib.sde_preprocess_u8(pi, H, W, pad, _need(out, "out_pad", shape=(H + 2 * pad, W + 2 * pad)),
                                _need(stats, "scratch", dtype=torch.uint8, shape=(nb,)),
                                _stream()), "sde_preprocess_u8")
    return out


def preprocess_u8_batch(imgs_u8, pad: int, out=None, stats=None):
    """u8 [N,H,W] -> zero-padded z-normalised f32 [N, H+2p, W+2p], all images per launch.
    stats: optional uint8 scratch tensor of N * preprocess_scratch_bytes(H, W) bytes."""
    N, H, W = imgs_u8.shape
    pi = _need(imgs_u8, "images", dtype=torch.uint8)
    nb = N * preprocess_scratch_bytes(H, W)
    if out is None:
        out = _empty((N, H + 2 * pad, W + 2 * pad), torch.float32, imgs_u8)
    if stats is None:
        stats = _empty((nb,), torch.uint8, imgs_u8)
    check(lib.sde_preprocess_u8_batch(pi, N, H, W, pad, _need(out, "out_pad", shape=(N, H + 2 * pad, W + 2 * pad)),
                                      _need(stats, "scratch", dtype=torch.uint8, shape=(nb,)),
                                      _stream()), "sde_preprocess_u8_batch")
    return out


# ----------------------------------------------------------------------------
# SGM and post-processing (process_functional.py:134-1088)
# ----------------------------------------------------------------------------
def sgm_penalties(img_u8, P1=2.3, P2=55.9, threshold=30, lamda=4, out=None):
    H, W = img_u8.shape
    pi = _need(img_u8, "image", dtype=torch.uint8)
    if out is None:
        out = _empty((H, W, 16), torch.float32, img_u8)
    check(lib.sde_sgm_penalties(pi, H, W, float(P1), float(P2), int(threshold), float(lamda),
                                _need(out, "penalties", shape=(H, W, 16)), _stream()), "sde_sgm_penalties")
    return out


def sgm_8path(cv_hwd, pen, S=None):
    H, W, D = cv_hwd.shape
    pc = _need(cv_hwd, "cost volume")
    pp = _need(pen, "penalties", shape=(H, W, 16))
    if S is None:
        S = torch.zeros((H, W, D), dtype=torch.float32, device=cv_hwd.device)
    # accumulates into S (the caller zeroes it, as the reference uploads np.zeros)
    check(lib.sde_sgm_8path(pc, pp, H, W, D, _need(S, "S", shape=(H, W, D)), _stream()), "sde_sgm_8path")
    return S


def sgm_8path_pair(cv_l, pen_l, S_l, cv_r=None, pen_r=None, S_r=None, accumulate=False, zero_du_penalties=False):
    """8-path SGM of both image sides, one launch per direction (sde_sgm_8path_pair).

    accumulate=False: S := the 8-path sum from zero (S need not be zeroed).
    zero_du_penalties=True: the penalties come from sgm_penalties (channels 0/1 zero) and
    the costs are finite -- direction DU is folded into the UD pass (same values)."""
    H, W, D = cv_l.shape
    args = [_need(cv_l, "cost volume"), _need(pen_l, "penalties", shape=(H, W, 16)), _need(S_l, "S", shape=(H, W, D))]
    if cv_r is None:
        args += [None, None, None]
    else:
        args += [_need(cv_r, "cost volume", shape=(H, W, D)), _need(pen_r, "penalties", shape=(H, W, 16)),
                 _need(S_r, "S", shape=(H, W, D))]
    flags = (_lib.SDE_SGM_ACCUMULATE if accumulate else 0) | \
        (_lib.SDE_SGM_ZERO_DU_PENALTIES if zero_du_penalties else 0)
    check(lib.sde_sgm_8path_pair(*args, H, W, D, flags, _stream()), "sde_sgm_8path_pair")
    return S_l, S_r


def sgm_8path_wta_pair(cv_l, pen_l, S_l, disp_l=None, cv_r=None, pen_r=None, S_r=None, disp_r=None,
                       accumulate=False, zero_du_penalties=False):
    """sgm_8path_pair + WTA (rule "d0") fused into the last direction (sde_sgm_8path_wta_pair):
    returns the disparity maps; S is left holding the first seven directions' sum."""
    H, W, D = cv_l.shape
    if disp_l is None:
        disp_l = _empty((H, W), torch.float32, cv_l)
    args = [_need(cv_l, "cost volume"), _need(pen_l, "penalties", shape=(H, W, 16)), _need(S_l, "S", shape=(H, W, D)),
            _need(disp_l, "disp", shape=(H, W))]
    if cv_r is None:
        args += [None, None, None, None]
    else:
        if disp_r is None:
            disp_r = _empty((H, W), torch.float32, cv_l)
        args += [_need(cv_r, "cost volume", shape=(H, W, D)), _need(pen_r, "penalties", shape=(H, W, 16)),
                 _need(S_r, "S", shape=(H, W, D)), _need(disp_r, "disp", shape=(H, W))]
    flags = (_lib.SDE_SGM_ACCUMULATE if accumulate else 0) | \
        (_lib.SDE_SGM_ZERO_DU_PENALTIES if zero_du_penalties else 0)
    check(lib.sde_sgm_8path_wta_pair(*args, H, W, D, flags, _stream()), "sde_sgm_8path_wta_pair")
    return disp_l, disp_r


def sgm_direction(cv_hwd, pen, direction: int, S):
    H, W, D = cv_hwd.shape
    check(lib.sde_sgm_direction(_need(cv_hwd, "cost volume"), _need(pen, "penalties", shape=(H, W, 16)), H, W, D,
                                int(direction), _need(S, "S", shape=(H, W, D)), _stream()), "sde_sgm_direction")
    return S


# ----------------------------------------------------------------------------
# Cross-based cost aggregation (build-defined; the reference has none)
# ----------------------------------------------------------------------------
CBCA_MAX_L1 = 32


def cbca_arms(img, L1=14, tau=0.02, out=None):
    """Cross arms of an f32 [H,W] device image (row-strided views allowed, e.g. the interior of the tower's
    padded input) -> int32-viewed u32 [H,W] packed l | r<<8 | u<<16 | d<<24 (sde_cbca_arms)."""
    if not isinstance(img, torch.Tensor) or img.dim() != 2 or img.dtype != torch.float32 or not img.is_cuda:
        raise ValueError("image must be a 2-D float32 GPU tensor")
    if img.stride(1) != 1:
        raise ValueError("image rows must be contiguous")
    H, W = img.shape
    if out is None:
        out = _empty((H, W), torch.int32, img)
    check(lib.sde_cbca_arms(img.data_ptr(), img.stride(0), H, W, int(L1), float(tau),
                            _need(out, "arms", dtype=torch.int32, shape=(H, W)), _stream()), "sde_cbca_arms")
    return out


def cbca_workspace_bytes(H, W):
    """Bytes of the aggregation workspace (column-major left-image arms, sde_cbca_workspace_bytes)."""
    return int(lib.sde_cbca_workspace_bytes(int(H), int(W)))


def _cbca_ws(ws, H, W, like):
    n = cbca_workspace_bytes(H, W)
    if ws is None:
        return _empty((n,), torch.uint8, like), n
    if not isinstance(ws, torch.Tensor) or not ws.is_cuda or ws.numel() * ws.element_size() < n:
        raise ValueError(f"cbca workspace must be a GPU tensor of at least {n} bytes")
    return ws, ws.numel() * ws.element_size()


def cbca(cv_hwd, arms_ref, arms_other, side="left", L1=14, iters=2, tmp=None, workspace=None):
    """In-place cross-based aggregation of an [H,W,D] volume (sde_cbca); tmp: same-size scratch."""
    H, W, D = cv_hwd.shape
    if tmp is None:
        tmp = torch.empty_like(cv_hwd)
    ws, nws = _cbca_ws(workspace, H, W, cv_hwd)
    sd = {"left": SDE_SIDE_LEFT, "right": SDE_SIDE_RIGHT}[side]
    check(lib.sde_cbca(_need(cv_hwd, "cost volume"), _need(tmp, "tmp", shape=(H, W, D)),
                       _need(arms_ref, "arms_ref", dtype=torch.int32, shape=(H, W)),
                       _need(arms_other, "arms_other", dtype=torch.int32, shape=(H, W)), H, W, D, sd, int(L1),
                       int(iters), ws.data_ptr(), nws, _stream()), "sde_cbca")
    return cv_hwd


def cbca_pair(cv_l, cv_r, arms_l, arms_r, L1=14, iters=2, tmp_l=None, tmp_r=None, workspace=None):
    """cbca(cv_l, arms_l, arms_r, "left") and cbca(cv_r, arms_r, arms_l, "right") for any two volumes
    (sde_cbca_pair), in place; tmp_l / tmp_r: same-size scratch, distinct from every volume."""
    H, W, D = cv_l.shape
    tmp_l = torch.empty_like(cv_l) if tmp_l is None else tmp_l
    tmp_r = torch.empty_like(cv_l) if tmp_r is None else tmp_r
    ws, nws = _cbca_ws(workspace, H, W, cv_l)
    check(lib.sde_cbca_pair(_need(cv_l, "cost volume"), _need(tmp_l, "tmp", shape=(H, W, D)),
                            _need(cv_r, "cost volume", shape=(H, W, D)), _need(tmp_r, "tmp", shape=(H, W, D)),
                            _need(arms_l, "arms_l", dtype=torch.int32, shape=(H, W)),
                            _need(arms_r, "arms_r", dtype=torch.int32, shape=(H, W)), H, W, D, int(L1), int(iters),
                            ws.data_ptr(), nws, _stream()), "sde_cbca_pair")
    return cv_l, cv_r


def cbca_lr(cv_l, cv_r, arms_l, arms_r, L1=14, iters=2, tmp=None, workspace=None):
    """The GPU path's pair (sde_cbca_lr): cv_l aggregated in place, then cv_r's valid voxels set to its
    shear cv_r[y, x, d] = cv_l[y, x + d, d] (x + d < W; the others untouched).  Equal to cbca_pair when
    cv_r's valid voxels are cv_l's shear (as cost_volume(..., right=True) writes them)."""
    H, W, D = cv_l.shape
    tmp = torch.empty_like(cv_l) if tmp is None else tmp
    ws, nws = _cbca_ws(workspace, H, W, cv_l)
    check(lib.sde_cbca_lr(_need(cv_l, "cost volume"), _need(cv_r, "cost volume", shape=(H, W, D)),
                          _need(tmp, "tmp", shape=(H, W, D)),
                          _need(arms_l, "arms_l", dtype=torch.int32, shape=(H, W)),
                          _need(arms_r, "arms_r", dtype=torch.int32, shape=(H, W)), H, W, D, int(L1), int(iters),
                          ws.data_ptr(), nws, _stream()), "sde_cbca_lr")
    return cv_l, cv_r


def cbca_reciprocals(n, device=None):
    """The fp64 reciprocals 1/(i+1), i < n, as the aggregation kernels compute them."""
    out = torch.empty((int(n),), dtype=torch.float64, device=device or torch.device("cuda"))
    check(lib.sde_cbca_reciprocals(out.data_ptr(), int(n), _stream()), "sde_cbca_reciprocals")
    return out


def lr_check(disp_l, disp_r, lrc_l=None, lrc_r=None):
    H, W = disp_l.shape
    if lrc_l is None:
        lrc_l = torch.zeros((H, W), dtype=torch.uint8, device=disp_l.device)
    if lrc_r is None:
        lrc_r = torch.zeros((H, W), dtype=torch.uint8, device=disp_l.device)
    check(lib.sde_lr_check(_need(disp_l, "disp_l"), _need(disp_r, "disp_r", shape=(H, W)), H, W,
                           _need(lrc_l, "lrc_l", dtype=torch.uint8, shape=(H, W)),
                           _need(lrc_r, "lrc_r", dtype=torch.uint8, shape=(H, W)), _stream()), "sde_lr_check")
    return lrc_l, lrc_r


def lrc_fill(disp_l, lrc_l, out=None):
    H, W = disp_l.shape
    if out is None:
        out = _empty((H, W), torch.float32, disp_l)
    check(lib.sde_lrc_fill(_need(disp_l, "disp_l"), _need(lrc_l, "lrc_l", dtype=torch.uint8, shape=(H, W)), H, W,
                           _need(out, "out", shape=(H, W)), _stream()), "sde_lrc_fill")
    return out


def median5(src, dst):
    H, W = src.shape
    check(lib.sde_median5(_need(src, "src"), H, W, _need(dst, "dst", shape=(H, W)), _stream()), "sde_median5")
    return dst
