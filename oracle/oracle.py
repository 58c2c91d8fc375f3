"""ctypes front-end of the C oracle (oracle/sde_oracle.c) plus NumPy restatements.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  Every function cites the
reference file:line it restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libsde_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build(force: bool = False) -> str:
    """Compile the C oracle with its Makefile (gcc, -ffp-contract=off)."""
    if force or not os.path.exists(_LIB_PATH) or \
            os.path.getmtime(_LIB_PATH) < os.path.getmtime(os.path.join(_HERE, "sde_oracle.c")):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.sdeo_set_threads.argtypes = [ctypes.c_int]
        L.sdeo_get_threads.restype = ctypes.c_int
        L.sdeo_np_sum_f32.restype = ctypes.c_float
        L.sdeo_np_sum_f32.argtypes = [_f32p, ctypes.c_long]
        L.sdeo_cost_volume_dhw.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 4 + [_f32p]
        L.sdeo_cost_volume_hwd.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 4 + [ctypes.c_float, _f32p, _f32p]
        L.sdeo_wta1_dhw.argtypes = [_f32p] + [ctypes.c_int] * 3 + [_f32p]
        L.sdeo_wta1_dhw.restype = ctypes.c_int
        L.sdeo_wta_hwd.argtypes = [_f32p] + [ctypes.c_int] * 3 + [_f32p]
        L.sdeo_wta_hwd.restype = ctypes.c_int
        L.sdeo_wta_sgm_hwd.argtypes = [_f32p] + [ctypes.c_int] * 3 + [_f32p]
        L.sdeo_cv_wta_shard.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 5 + [_f32p, _i32p]
        L.sdeo_sgm_penalties.argtypes = [_u8p, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                                         ctypes.c_double, ctypes.c_long, ctypes.c_double, _f32p]
        L.sdeo_sgm_direction.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 4 + [_f32p]
        L.sdeo_sgm_8path.argtypes = [_f32p, _f32p] + [ctypes.c_int] * 3 + [_f32p]
        L.sdeo_lr_check.argtypes = [_f32p, _f32p, ctypes.c_int, ctypes.c_int, _u8p, _u8p]
        L.sdeo_lrc_fill.argtypes = [_f32p, _u8p, ctypes.c_int, ctypes.c_int, _f32p]
        L.sdeo_median5.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, _f32p]
        L.sdeo_tower_forward.argtypes = [_f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(_f32p), ctypes.POINTER(_f32p), _f32p]
        _u32p = ctypes.POINTER(ctypes.c_uint32)
        L.sdeo_cbca_arms.argtypes = [_f32p, ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                                     _u32p]
        L.sdeo_cbca.argtypes = [_f32p, _f32p, _u32p, _u32p] + [ctypes.c_int] * 6
        L.sdeo_cbca_lr.argtypes = [_f32p, _f32p, _f32p, _u32p, _u32p] + [ctypes.c_int] * 5
        L.sdeo_cbca_seg.restype = ctypes.c_int
        _lib = L
        L.sdeo_set_threads(int(os.environ.get("SDE_ORACLE_THREADS", min(16, os.cpu_count() or 1))))
    return _lib


def set_threads(n: int) -> None:
    """OpenMP threads for the oracle's parallel loops (bit-identical results for any count)."""
    lib().sdeo_set_threads(int(n))


def get_threads() -> int:
    return int(lib().sdeo_get_threads())


def _p(a, t=_f32p):
    return a.ctypes.data_as(t)


def _c32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


# --------------------------------------------------------------------------
# CPU path: process_functional.py:48-113
# --------------------------------------------------------------------------
def compute_cost_volume(featuresl, featuresr, ndisp):
    """compute_cost_volume (process_functional.py:48-73) -> f32 [D,H,W], bit-exact."""
    fl, fr = _c32(featuresl), _c32(featuresr)
    H, W, C = fl.shape
    out = np.empty((ndisp, H, W), np.float32)
    lib().sdeo_cost_volume_dhw(_p(fl), _p(fr), H, W, C, ndisp, _p(out))
    return out


def cost_volume_hwd(featuresl, featuresr, ndisp, invalid=1.0, right=True):
    """GPU-path layout [H,W,D] (process_functional.py:120-131, fill :1111) with CPU numerics."""
    fl, fr = _c32(featuresl), _c32(featuresr)
    H, W, C = fl.shape
    outl = np.empty((H, W, ndisp), np.float32)
    outr = np.empty((H, W, ndisp), np.float32) if right else None
    lib().sdeo_cost_volume_hwd(_p(fl), _p(fr), H, W, C, ndisp, invalid, _p(outl),
                               _p(outr) if right else None)
    return (outl, outr) if right else outl


def WTA1(cv):
    """WTA1 (process_functional.py:96-113) on [D,H,W]."""
    cv = _c32(cv)
    D, H, W = cv.shape
    out = np.empty((H, W), np.float32)
    bad = lib().sdeo_wta1_dhw(_p(cv), D, H, W, _p(out))
    assert bad == 0
    return out


def WTA(cv):
    """WTA (process_functional.py:76-93) on [H,W,D]."""
    cv = _c32(cv)
    H, W, D = cv.shape
    out = np.empty((H, W), np.float32)
    bad = lib().sdeo_wta_hwd(_p(cv), H, W, D, _p(out))
    assert bad == 0
    return out


def wta_sgm(S):
    """WTA_and_SupixelRefinement_kernel (process_functional.py:800-837) on [H,W,D]."""
    S = _c32(S)
    H, W, D = S.shape
    out = np.empty((H, W), np.float32)
    lib().sdeo_wta_sgm_hwd(_p(S), H, W, D, _p(out))
    return out


def cv_wta_shard(featuresl, featuresr, d0, d1):
    """First-min over disparities [d0,d1) of the CPU-path costs: (min f32 [H,W], argmin i32 [H,W])."""
    fl, fr = _c32(featuresl), _c32(featuresr)
    H, W, C = fl.shape
    mn = np.empty((H, W), np.float32)
    am = np.empty((H, W), np.int32)
    lib().sdeo_cv_wta_shard(_p(fl), _p(fr), H, W, C, d0, d1, _p(mn), _p(am, _i32p))
    return mn, am


def np_sum_f32(a):
    a = _c32(a).ravel()
    return np.float32(lib().sdeo_np_sum_f32(_p(a), a.size))


# --------------------------------------------------------------------------
# GPU path restatements: process_functional.py:134-1088 (parity unpinned)
# --------------------------------------------------------------------------
def sgm_penalties(image_u8, P1=2.3, P2=55.9, threshold=30, lamda=4):
    """sgm_penelty_kernel (process_functional.py:134-262) -> f32 [H,W,16]."""
    img = np.ascontiguousarray(image_u8, dtype=np.uint8)
    H, W = img.shape
    pen = np.empty((H, W, 16), np.float32)
    lib().sdeo_sgm_penalties(_p(img, _u8p), H, W, float(P1), float(P2), int(threshold), float(lamda), _p(pen))
    return pen


SGM_DIRECTIONS = ("UD", "DU", "LR", "RL", "UD_LR", "DU_LR", "UD_RL", "DU_RL")


def sgm_direction(cv_hwd, pen, direction, S=None):
    """One SGM_*_kernel pass (process_functional.py:346-797) for one side; accumulates into S."""
    cv = _c32(cv_hwd)
    pen = _c32(pen)
    H, W, D = cv.shape
    if S is None:
        S = np.zeros((H, W, D), np.float32)
    assert S.flags.c_contiguous and S.dtype == np.float32
    d = SGM_DIRECTIONS.index(direction) if isinstance(direction, str) else int(direction)
    lib().sdeo_sgm_direction(_p(cv), _p(pen), H, W, D, d, _p(S))
    return S


def sgm_8path(cv_hwd, pen, S=None):
    """All 8 directions in launch order (process_functional.py:1166-1203) for one side -> S f32 [H,W,D].

    S: optional initial S (accumulated into, in place); zeros as the reference uploads by default."""
    cv = _c32(cv_hwd)
    pen = _c32(pen)
    H, W, D = cv.shape
    if H < 2 or W < 2:
        raise ValueError("SGM needs H >= 2 and W >= 2 (the reference indexes out of bounds otherwise)")
    if S is None:
        S = np.zeros((H, W, D), np.float32)
    assert S.dtype == np.float32 and S.shape == cv.shape and S.flags.c_contiguous
    lib().sdeo_sgm_8path(_p(cv), _p(pen), H, W, D, _p(S))
    return S


def lr_check(dl, dr):
    """is_error_match_kernel (process_functional.py:977-1000) -> (lrc_l, lrc_r) u8, zero-initialised."""
    dl, dr = _c32(dl), _c32(dr)
    H, W = dl.shape
    a = np.zeros((H, W), np.uint8)
    b = np.zeros((H, W), np.uint8)
    lib().sdeo_lr_check(_p(dl), _p(dr), H, W, _p(a, _u8p), _p(b, _u8p))
    return a, b


def lrc_fill(dl, lrc_l):
    """LRC_kernel left output (process_functional.py:1003-1088)."""
    dl = _c32(dl)
    f = np.ascontiguousarray(lrc_l, dtype=np.uint8)
    H, W = dl.shape
    out = np.empty((H, W), np.float32)
    lib().sdeo_lrc_fill(_p(dl), _p(f, _u8p), H, W, _p(out))
    return out


def median5(src, dst_init):
    """Median_Filter_kernel (process_functional.py:840-879): interior only; border keeps dst_init."""
    src = _c32(src)
    out = np.array(dst_init, dtype=np.float32, copy=True)
    H, W = src.shape
    lib().sdeo_median5(_p(src), H, W, _p(out))
    return out


def tower_forward(img_pad, weights, biases):
    """MC-CNN-fast branch (mc_cnn_brunch.py:31-48,70-92) in fp64 -> f32 [H,W,nf].

    img_pad: f32 [H+2L, W+2L] zero-padded image; weights[l]: HWIO [3,3,Cin,nf]; biases[l]: [nf].
    """
    img = _c32(img_pad)
    Hp, Wp = img.shape
    L = len(weights)
    nf = weights[0].shape[-1]
    ws = [_c32(w) for w in weights]
    bs = [_c32(b) for b in biases]
    wp = (_f32p * L)(*[_p(w) for w in ws])
    bp = (_f32p * L)(*[_p(b) for b in bs])
    out = np.empty((Hp - 2 * L, Wp - 2 * L, nf), np.float32)
    lib().sdeo_tower_forward(_p(img), Hp, Wp, L, nf, wp, bp, _p(out))
    return out


def znorm(image_f32):
    """Per-image z-normalisation exactly as match_single.py:40-41 (NumPy float32)."""
    x = np.asarray(image_f32, dtype=np.float32)
    return (x - np.mean(x, axis=(0, 1))) / np.std(x, axis=(0, 1))


def pad_image(image, patch=11):
    """compute_feature's zero padding (process_functional.py:13-19) -> f32 [H+p-1, W+p-1]."""
    x = np.asarray(image, dtype=np.float32)
    if x.ndim == 3:
        x = x[..., 0]
    H, W = x.shape
    out = np.zeros((H + patch - 1, W + patch - 1), np.float32)
    s = (patch - 1) // 2
    out[s:s + H, s:s + W] = x
    return out


# --------------------------------------------------------------------------
# Cross-based cost aggregation: BUILD-DEFINED (absent in the reference,
# SURVEY.md sec. 0.3) -- parity unpinned; definition in sde_oracle.c.
# --------------------------------------------------------------------------
def cbca_arms(img, L1=14, tau=0.02):
    """Cross arms of an f32 [H,W] image -> u32 [H,W] packed left | right<<8 | up<<16 | down<<24."""
    im = _c32(img)
    H, W = im.shape
    out = np.empty((H, W), np.uint32)
    lib().sdeo_cbca_arms(_p(im), W, H, W, int(L1), float(tau), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    return out


def cbca_seg():
    """Segment length of the CBCA definition (SDE_CBCA_SEG)."""
    return int(lib().sdeo_cbca_seg())


def _arms(a, L1):
    a = np.ascontiguousarray(a, dtype=np.uint32)
    M = max(int(L1) - 1, 0)
    for k in range(4):   # the definition's windows reach at most M = L1 - 1 positions per arm
        if ((a >> (8 * k)) & 255).max(initial=0) > M:
            raise ValueError(f"arms exceed L1 - 1 = {M}")
    return a


def cbca(cv_hwd, arms_ref, arms_other, side="left", iters=1, L1=14):
    """iters x (horizontal then vertical cross-support mean) of an [H,W,D] volume (new array);
    definition v2 (sde_oracle.c): left coordinates, segmented prefix chains, invalid voxels kept."""
    cv = np.array(cv_hwd, dtype=np.float32, order="C", copy=True)
    H, W, D = cv.shape
    tmp = np.empty_like(cv)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    a, b = _arms(arms_ref, L1), _arms(arms_other, L1)
    lib().sdeo_cbca(_p(cv), _p(tmp), a.ctypes.data_as(u32p), b.ctypes.data_as(u32p), H, W, D,
                    1 if side == "left" else 2, int(L1), int(iters))
    return cv


def cbca_lr(cv_l, cv_r, arms_l, arms_r, iters=1, L1=14):
    """sde_cbca_lr: the left volume aggregated, the right one's valid voxels set to its shear
    (invalid ones kept).  Returns (left, right) as new arrays."""
    cl = np.array(cv_l, dtype=np.float32, order="C", copy=True)
    cr = np.array(cv_r, dtype=np.float32, order="C", copy=True)
    H, W, D = cl.shape
    tmp = np.empty_like(cl)
    u32p = ctypes.POINTER(ctypes.c_uint32)
    a, b = _arms(arms_l, L1), _arms(arms_r, L1)
    lib().sdeo_cbca_lr(_p(cl), _p(cr), _p(tmp), a.ctypes.data_as(u32p), b.ctypes.data_as(u32p), H, W, D,
                       int(L1), int(iters))
    return cl, cr
