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


def support(ref, oth, y, x, d, side):
    W = ref.shape[1]
    o = x - d if side == "left" else x + d
    if not 0 <= o < W:
        return [0, 0, 0, 0]
    return [min((int(ref[y, x]) >> (8 * k)) & 255, (int(oth[y, o]) >> (8 * k)) & 255) for k in range(4)]


def cbca_literal(cv, ref, oth, side, iters):
    H, W, D = cv.shape
    cur = cv.copy()
    for _ in range(iters):
        T = np.zeros_like(cur)
        for y in range(H):
            for d in range(D):
                P = [0.0]
                for x in range(W):
                    P.append(P[-1] + float(cur[y, x, d]))          # Python float = IEEE fp64
                for x in range(W):
                    a = support(ref, oth, y, x, d, side)
                    T[y, x, d] = np.float32(P[x + a[1] + 1] - P[x - a[0]])
        nxt = np.zeros_like(cur)
        for x in range(W):
            for d in range(D):
                Q, N = [0.0], [0]
                for y in range(H):
                    b = support(ref, oth, y, x, d, side)
                    Q.append(Q[-1] + float(T[y, x, d]))
                    N.append(N[-1] + b[0] + b[1] + 1)
                for y in range(H):
                    a = support(ref, oth, y, x, d, side)
                    nxt[y, x, d] = np.float32((Q[y + a[3] + 1] - Q[y - a[2]]) / float(N[y + a[3] + 1] - N[y - a[2]]))
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
    got = oracle.cbca(cv, ref, oth, side, iters)
    assert got.tobytes() == cbca_literal(cv, ref, oth, side, iters).tobytes()


def test_cbca_properties():
    rng = np.random.default_rng(3)
    H, W, D = 12, 17, 6
    cv = rng.standard_normal((H, W, D)).astype(np.float32)
    flat = np.zeros((H, W), np.float32)
    zero = oracle.cbca_arms(flat, 14, 0.0)                 # tau = 0: no arms -> identity (up to the prefix
    np.testing.assert_allclose(oracle.cbca(cv, zero, zero, "left", 3), cv, rtol=1e-7, atol=1e-12)  # rounding)
    assert oracle.cbca(cv, zero, zero, "left", 0).tobytes() == cv.tobytes()
    full = oracle.cbca_arms(flat, 64, 1.0)                 # flat image, long arms: support = whole image
    out = oracle.cbca(cv, full, full, "left", 1)
    for d in range(D):
        # left-referenced: voxels with x >= d average over the region x' >= d; x < d stays as is
        np.testing.assert_allclose(out[:, d:, d], cv[:, d:, d].mean(), rtol=2e-5, atol=2e-6)
        np.testing.assert_allclose(out[:, :d, d], cv[:, :d, d], rtol=1e-7, atol=1e-12)
