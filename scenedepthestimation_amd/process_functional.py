"""Drop-in replacement of the reference's ``process_functional`` function API.

Same names, argument meaning, return types and error behaviour as
WHDY/SceneDepthEstimation process_functional.py, which the entry points
star-import (match_single.py:9, match.py:10, match_single_ui.py:9):

  compute_feature(left_image, right_image, patch_height, patch_width,
                  num_of_feature_maps, checkpoint)          :11-45
  compute_cost_volume(featuresl, featuresr, ndisp)           :48-73
  WTA(left_cost_volume)                                      :76-93
  WTA1(left_cost_volume)                                     :96-113
  disparity_compute_by_gpu(imagel, imager, featuresl,
                           featuresr, detail_time)           :1093-1267

NumPy arrays in, new NumPy arrays out; ``detail_time`` is updated in place and
returned.  Every computation runs in libsde.so's HIP kernels on the current
GPU (the reference pins TF to GPU 0 and Numba to visible GPU 1; here one device
does both and no host round trip sits between the stages of
``disparity_compute_by_gpu``).  There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np
import torch

from . import mc_cnn, ops
from .pipeline import StereoMatcher

__all__ = ["compute_feature", "compute_cost_volume", "WTA", "WTA1", "disparity_compute_by_gpu"]


def _device():
    if not torch.cuda.is_available():
        raise RuntimeError("scenedepthestimation_amd needs a ROCm GPU (libsde.so has no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def _to_dev(a, dtype=np.float32):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=dtype)).to(_device())


def compute_feature(left_image, right_image, patch_height, patch_width, num_of_feature_maps, checkpoint):
    """MC-CNN features of both images (process_functional.py:11-45) -> (fl, fr) f32 [H,W,nf].

    Images are the normalised float images the entry points build ([H,W,1] or [H,W]).
    `checkpoint`: weights dict / .npz / .safetensors / 'synthetic[:seed]' / None (see mc_cnn.load_weights).
    """
    if patch_height != patch_width or patch_height % 2 != 1:
        raise ValueError("the MC-CNN-fast branch uses square odd patches (11x11 in the reference)")
    nlayers = patch_height // 2                         # process_functional.py:23
    if num_of_feature_maps != 64:
        raise ValueError("libsde's tower kernels are built for 64 feature maps (the reference's setting)")
    li = np.asarray(left_image, np.float32)
    ri = np.asarray(right_image, np.float32)
    li = li[..., 0] if li.ndim == 3 else li
    ri = ri[..., 0] if ri.ndim == 3 else ri
    if li.shape != ri.shape:
        raise ValueError("left and right images differ in shape")
    H, W = li.shape
    weights = mc_cnn.load_weights(checkpoint, nlayers)
    m = StereoMatcher(H, W, 1, weights=weights, nlayers=nlayers, nf=num_of_feature_maps, device=_device())
    pad = (patch_height - 1) // 2                       # zero padding, process_functional.py:13-19
    for i, img in enumerate((li, ri)):
        buf = np.zeros((H + 2 * pad, W + 2 * pad), np.float32)
        buf[pad:pad + H, pad:pad + W] = img
        m.img_pad[i].copy_(torch.from_numpy(buf))
    fl, fr = m.features_from_padded()
    return fl.cpu().numpy(), fr.cpu().numpy()


def compute_cost_volume(featuresl, featuresr, ndisp):
    """Left cost volume f32 [D,H,W] (process_functional.py:48-73), bit-identical to the reference."""
    fl, fr = _to_dev(featuresl), _to_dev(featuresr)
    if fl.dim() != 3 or fl.shape != fr.shape:
        raise ValueError("features must be matching [H,W,C] arrays")
    return ops.cost_volume(fl, fr, int(ndisp), layout="DHW").cpu().numpy()


def _checked(disp):
    d = disp.cpu().numpy()
    assert (d >= 0).all()            # the reference asserts min_disparity >= 0 (:89, :109)
    return d


def WTA(left_cost_volume):
    """First-min disparity of an [H,W,D] volume (process_functional.py:76-93) -> f32 [H,W]."""
    return _checked(ops.wta(_to_dev(left_cost_volume), layout="HWD", rule="inf"))


def WTA1(left_cost_volume):
    """First-min disparity of a [D,H,W] volume (process_functional.py:96-113) -> f32 [H,W]."""
    return _checked(ops.wta(_to_dev(left_cost_volume), layout="DHW", rule="inf"))


def disparity_compute_by_gpu(imagel, imager, featuresl, featuresr, detail_time, ndisp=128):
    """GPU path (process_functional.py:1093-1267): cost volume [H,W,D] (L, R; 1.0 fill),
    SGM penalties, 8-path SGM, WTA, LR check + LRC fill, 5x5 median.

    Returns (disparity_left, disparity_right, detail_time); detail_time slots as the
    reference: [1] cost volume, [3] SGM, [4] WTA, [5] LR check, [6] filtering (seconds).
    ``ndisp`` defaults to the reference's hard-coded 128 (:1111).
    """
    assert imagel.shape == imager.shape                   # :1097
    H, W = imagel.shape[0:2]
    fl, fr = _to_dev(featuresl), _to_dev(featuresr)
    il = _to_dev(imagel, np.uint8)
    ir = _to_dev(imager, np.uint8)
    if fl.shape[:2] != (H, W):
        raise ValueError("features and images differ in size")
    m = StereoMatcher.__new__(StereoMatcher)
    m.H, m.W, m.D, m.device = H, W, int(ndisp), fl.device
    m.sgm_bufs = None
    m.cbca_iters = 0          # the reference has no aggregation stage
    timings = {}
    dl, dr = m.sgm_path(fl=fl, fr=fr, img_l=il, img_r=ir, timings=timings)
    for slot, key in ((1, "cost_volume"), (3, "sgm"), (4, "wta"), (5, "lrc"), (6, "filter")):
        detail_time[slot] += timings.get(key, 0.0)
    return dl.cpu().numpy(), dr.cpu().numpy(), detail_time

