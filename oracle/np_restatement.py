"""NumPy restatement of the reference's CPU path -- TEST INFRASTRUCTURE / CPU BASELINE ONLY.

The same NumPy expressions as process_functional.py:48-73 (compute_cost_volume: one
np.multiply + np.sum(axis=-1) over an (H, W-d, C) temporary per disparity, then the sign
flip) and WTA1 (process_functional.py:96-113) two ways: ``wta1_loop``, the reference's own
form -- a Python loop over pixels with a scalar scan over d, which is what match_single.py:51-53
actually runs and where most of its CPU time goes -- and ``wta1_np``, np.argmin over the
disparity axis (the same first minimum when no cost is NaN; the golden vectors pin both).
Single-threaded (NumPy runs these element-wise kernels on one core).  bench.py times both
beside the C port, labelled apart.
"""
from __future__ import annotations

import numpy as np


def compute_cost_volume_np(featuresl, featuresr, ndisp):
    """process_functional.py:48-73 -> f32 [D, H, W]: cv[d, :, d:] = -sum_c fl[:, d:] * fr[:, :W-d]."""
    fl = np.asarray(featuresl, np.float32)
    fr = np.asarray(featuresr, np.float32)
    H, W = fl.shape[:2]
    cv = np.zeros((ndisp, H, W), np.float32)
    for d in range(min(ndisp, W)):
        cv[d, :, d:] = np.sum(np.multiply(fl[:, d:], fr[:, :W - d]), axis=-1)
    return -1 * cv          # (the reference's :72; -0.0 where nothing was computed)


def wta1_loop(cost_volume):
    """process_functional.py:96-113 as the reference executes it: per pixel, a scalar scan over d
    keeping the first strict minimum (and the reference's assert that one was found)."""
    cv = np.asarray(cost_volume, np.float32)
    D, H, W = cv.shape
    out = np.empty((H, W), np.float32)
    for h in range(H):
        for w in range(W):
            best, arg = float("inf"), -1
            for d in range(D):
                v = cv[d, h, w]
                if v < best:
                    best, arg = v, d
            assert arg >= 0
            out[h, w] = arg
    return out


def wta1_np(cost_volume):
    """process_functional.py:96-113 on [D, H, W] -> f32 [H, W] (first minimum over d)."""
    return np.argmin(cost_volume, axis=0).astype(np.float32)
