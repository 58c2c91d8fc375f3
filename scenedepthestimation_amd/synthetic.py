"""Seeded synthetic stereo inputs: no datasets are available offline.

Left  = uniform u8 texture, 3x3 box-blurred (seed).
Right = left warped by a piecewise-constant disparity field of vertical bands
        in [0, D-1] (seed + 1); pixels whose source falls outside the image are
        filled from the RNG.  Convention of the reference's cost volume: left
        pixel x matches right pixel x - d (process_functional.py:58).
"""
from __future__ import annotations

import numpy as np


def texture(H: int, W: int, rng) -> np.ndarray:
    raw = rng.integers(0, 256, (H + 2, W + 2)).astype(np.float32)
    blur = sum(raw[dy:dy + H, dx:dx + W] for dy in range(3) for dx in range(3)) / 9.0
    return np.clip(np.rint(blur), 0, 255).astype(np.uint8)


def band_disparity(H: int, W: int, D: int, rng, band: int = 64) -> np.ndarray:
    nb = (W + band - 1) // band
    vals = rng.integers(0, max(D, 1), nb)
    return np.repeat(vals, band)[:W][None, :].repeat(H, 0).astype(np.int32)


def stereo_pair(H: int, W: int, D: int, seed: int = 0):
    """-> (left u8 [H,W], right u8 [H,W], ground-truth left disparity int32 [H,W])."""
    rng = np.random.default_rng(seed)
    left = texture(H, W, rng)
    gt = band_disparity(H, W, D, np.random.default_rng(seed + 1))
    right = rng.integers(0, 256, (H, W)).astype(np.uint8)
    xs = np.arange(W)[None, :].repeat(H, 0)
    ys = np.arange(H)[:, None].repeat(W, 1)
    # right[y, x - d(x)] = left[y, x]
    xr = xs - gt
    ok = xr >= 0
    right[ys[ok], xr[ok]] = left[ys[ok], xs[ok]]
    return left, right, gt


def features(H: int, W: int, C: int = 64, seed: int = 0) -> np.ndarray:
    """L2-normalised N(0,1) features (cost-volume microbenchmarks)."""
    x = np.random.default_rng(seed).standard_normal((H, W, C)).astype(np.float32)
    n = np.sqrt((x.astype(np.float64) ** 2).sum(-1, keepdims=True))
    return (x / np.maximum(n, 1e-12)).astype(np.float32)
