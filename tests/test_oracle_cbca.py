"""CPU: the C restatement of cross-based aggregation (oracle/sde_oracle.c sdeo_cbca_*) against an
independent literal Python restatement, plus the definition's structural properties.

CBCA is BUILD-DEFINED: the reference has none -- parity unpinned vs the reference."""
import numpy as np
import pytest

from oracle import oracle


def arms_literal(img, L1, tau):
    H, W = img.shape
    out = np.zeros((H, W), np.uint32)
    for y in range(H):
        for x in range(W):
            packed = 0
            for k, (dy, dx) in enumerate(((0, -1), (0, 1), (-1, 0), (1, 0))):
                n = 0
                while n + 1 <= L1 - 1:
                    yy, xx = y + (n + 1) * dy, x + (n + 1) * dx
                    if not (0 <= yy < H and 0 <= xx < W):
                        break
                    if not (abs(np.float32(img[y, x]) - np.float32(img[yy, xx])) < np.float32(tau)):
                        break
                    n += 1
                packed |= n << (8 * k)
            out[y, x] = packed
    return out


SEG = 256   # SDE_CBCA_SEG


def support(ref, oth, y, x, d, side):
    """Support arms of voxel (y, x, d) in its own coordinates (None if invalid)."""
    W = ref.shape[1]
    o = x - d if side == "left" else x + d
    if not 0 <= o < W:
        return None
    return [min((int(ref[y, x]) >> (8 * k)) & 255, (int(oth[y, o]) >> (8 * k)) & 255) for k in range(4)]


def cbca_literal(cv, ref, oth, side, iters, L1):
    """Definition v2 stated voxel by voxel in the volume's OWN coordinates: a right-referenced
    voxel x' sits at left coordinate q = x' + d, which fixes its segment and chain base."""
    H, W, D = cv.shape
    M = L1 - 1
    lq = (lambda x, d: x) if side == "left" else (lambda x, d: x + d)     # left coordinate
    xq = (lambda q, d: q) if side == "left" else (lambda q, d: q - d)     # back to own coordinate
    cur = cv.copy()
    for _ in range(iters):
        T = cur.copy()                                       # invalid voxels pass through
        for y in range(H):
            for d in range(D):
                for x in range(W):
                    a = support(ref, oth, y, x, d, side)
                    if a is None:
                        continue
                    q = lq(x, d)
                    k = q // SEG
                    b = max(k * SEG - M, d)                  # chain base (left coordinates)
                    P = {b - 1: 0.0}
                    for i in range(b, q + a[1] + 1):
                        P[i] = P[i - 1] + float(cur[y, xq(i, d), d])   # Python float = IEEE fp64
                    T[y, x, d] = np.float32(P[q + a[1]] - P[q - a[0] - 1])
        nxt = T.copy()
        for x in range(W):
            for d in range(D):
                for y in range(H):
                    a = support(ref, oth, y, x, d, side)
                    if a is None:
                        nxt[y, x, d] = cur[y, x, d]
                        continue
                    k = y // SEG
                    b = max(k * SEG - M, 0)
                    Q, N = {b - 1: 0.0}, {b - 1: 0}
                    for i in range(b, y + a[3] + 1):
                        s = support(ref, oth, i, x, d, side)
                        Q[i] = Q[i - 1] + float(T[i, x, d])
                        N[i] = N[i - 1] + s[0] + s[1] + 1
                    cnt = N[y + a[3]] - N[y - a[2] - 1]
                    nxt[y, x, d] = np.float32((Q[y + a[3]] - Q[y - a[2] - 1]) * (1.0 / float(cnt)))
        cur = nxt
    return cur


def _images(rng, H, W):
    # piecewise-flat images so arms take every length from 0 to L1-1
    base = rng.integers(0, 4, (H, W)).astype(np.float32) * 0.05
    return np.repeat(base[:, ::3], 3, axis=1)[:, :W] + rng.standard_normal((H, W)).astype(np.float32) * 0.003


@pytest.mark.parametrize("L1,tau", [(4, 0.02), (6, 0.06), (1, 1.0)])
def test_arms_match_literal(L1, tau):
    rng = np.random.default_rng(L1)
    img = _images(rng, 9, 13)
    got = oracle.cbca_arms(img, L1, tau)
    assert np.array_equal(got, arms_literal(img, L1, tau))
    assert ((got & 255) <= max(L1 - 1, 0)).all()


@pytest.mark.parametrize("side,iters", [("left", 1), ("right", 2), ("left", 0)])
def test_cbca_matches_literal(side, iters):
    rng = np.random.default_rng(7)
    H, W, D = 7, 11, 5
    il, ir = _images(rng, H, W), _images(rng, H, W)
    al, ar = oracle.cbca_arms(il, 5, 0.03), oracle.cbca_arms(ir, 5, 0.03)
    ref, oth = (al, ar) if side == "left" else (ar, al)
    cv = rng.standard_normal((H, W, D)).astype(np.float32)
    got = oracle.cbca(cv, ref, oth, side, iters, L1=5)
    assert got.tobytes() == cbca_literal(cv, ref, oth, side, iters, 5).tobytes()


@pytest.mark.parametrize("side,H,W", [("left", 5, 300), ("right", 5, 300), ("left", 290, 6), ("right", 290, 6)])
def test_cbca_segments_match_literal(side, H, W):
    """Lines longer than one segment (SDE_CBCA_SEG = 256): chains restart at kS - M."""
    assert oracle.cbca_seg() == SEG
    rng = np.random.default_rng(11)
    D = 3
    il, ir = _images(rng, H, W), _images(rng, H, W)
    al, ar = oracle.cbca_arms(il, 6, 0.06), oracle.cbca_arms(ir, 6, 0.06)
    ref, oth = (al, ar) if side == "left" else (ar, al)
    cv = (rng.standard_normal((H, W, D)) * 3 + 20).astype(np.float32)   # far from 0: rounding matters
    got = oracle.cbca(cv, ref, oth, side, 1, L1=6)
    assert got.tobytes() == cbca_literal(cv, ref, oth, side, 1, 6).tobytes()


def _shear(cl):
    """Right-referenced volume of a left one: R(y, x', d) = L(y, x'+d, d), invalid voxels 1.0."""
    H, W, D = cl.shape
    cr = np.ones_like(cl)
    for d in range(D):
        cr[:, :W - d, d] = cl[:, d:, d]
    return cr


@pytest.mark.parametrize("L1,iters", [(14, 2), (5, 1)])
def test_cbca_right_is_shear_of_left(L1, iters):
    """CBCA(R) = shear(CBCA(L)) exactly when R = shear(L): the one support of both volumes, and the
    pair entry point (left aggregated, right sheared) equals aggregating both."""
    rng = np.random.default_rng(5)
    H, W, D = 9, 270, 12
    il, ir = _images(rng, H, W), _images(rng, H, W)
    al, ar = oracle.cbca_arms(il, L1, 0.03), oracle.cbca_arms(ir, L1, 0.03)
    cl = (rng.standard_normal((H, W, D)) + 5).astype(np.float32)
    for d in range(D):
        cl[:, :d, d] = 1.0                                  # the GPU path's invalid fill
    cr = _shear(cl)
    left = oracle.cbca(cl, al, ar, "left", iters, L1=L1)
    right = oracle.cbca(cr, ar, al, "right", iters, L1=L1)
    assert right.tobytes() == _shear(left).tobytes()
    lr_l, lr_r = oracle.cbca_lr(cl, cr, al, ar, iters, L1=L1)
    assert lr_l.tobytes() == left.tobytes() and lr_r.tobytes() == right.tobytes()


def test_cbca_properties():
    rng = np.random.default_rng(3)
    H, W, D = 12, 17, 6
    cv = rng.standard_normal((H, W, D)).astype(np.float32)
    flat = np.zeros((H, W), np.float32)
    zero = oracle.cbca_arms(flat, 14, 0.0)                 # tau = 0: no arms -> identity (up to the prefix
    np.testing.assert_allclose(oracle.cbca(cv, zero, zero, "left", 3), cv, rtol=1e-7, atol=1e-12)  # rounding)
    assert oracle.cbca(cv, zero, zero, "left", 0).tobytes() == cv.tobytes()
    full = oracle.cbca_arms(flat, 32, 1.0)                 # flat image, long arms: support = whole image
    out = oracle.cbca(cv, full, full, "left", 1, L1=32)
    for d in range(D):
        # left-referenced: voxels with x >= d average over the region x' >= d; x < d stays as is
        np.testing.assert_allclose(out[:, d:, d], cv[:, d:, d].mean(), rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(out[:, :d, d], cv[:, :d, d], rtol=1e-7, atol=1e-12)
