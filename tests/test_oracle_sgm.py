"""CPU: the C oracle's SGM agrees bit-for-bit with the literal restatement of the Numba kernels."""
import numpy as np
import pytest

from sgm_literal import sgm_8path_literal


def _case(seed, H, W, D, invalid_frac=0.2):
    rng = np.random.default_rng(seed)
    cv = (rng.standard_normal((H, W, D)) * 0.5).astype(np.float32)
    cv[rng.random((H, W, D)) < invalid_frac] = 1.0
    img = rng.integers(0, 256, (H, W)).astype(np.uint8)
    img[rng.random((H, W)) < 0.3] = 128        # runs of equal intensity -> both penalty branches
    return cv, img


@pytest.mark.parametrize("H,W,D", [(5, 6, 8), (7, 4, 12), (2, 3, 8), (3, 2, 4), (4, 9, 16), (6, 6, 128)])
def test_sgm_oracle_matches_literal(oracle, H, W, D):
    cv, img = _case(H * 100 + W * 10 + D, H, W, D)
    pen = oracle.sgm_penalties(img)
    S_lit = sgm_8path_literal(cv, pen)
    S_or = oracle.sgm_8path(cv, pen)
    assert S_or.tobytes() == S_lit.tobytes()


@pytest.mark.parametrize("H,W,D", [(5, 6, 8), (4, 9, 16), (6, 5, 128), (3, 7, 4)])
def test_sgm_oracle_matches_literal_nonfinite(oracle, H, W, D):
    """NaN / +-inf costs: the binary-min order and the per-lane minima decide where they propagate."""
    cv, img = _case(H * 7 + W * 3 + D, H, W, D)
    rng = np.random.default_rng(D)
    cv[rng.random(cv.shape) < 0.04] = np.nan
    cv[rng.random(cv.shape) < 0.04] = np.inf
    cv[rng.random(cv.shape) < 0.02] = -np.inf
    cv[1, :, :4] = np.nan                     # a whole first lane NaN on one row
    pen = oracle.sgm_penalties(img)
    S_lit = sgm_8path_literal(cv, pen)
    S_or = oracle.sgm_8path(cv, pen)
    # NaN payloads are not part of the contract: compare with NaNs canonicalised
    assert np.array_equal(np.isnan(S_or), np.isnan(S_lit))
    assert np.nan_to_num(S_or, nan=7.0).tobytes() == np.nan_to_num(S_lit, nan=7.0).tobytes()
    # the per-lane minima matter: some lane saw a NaN the others ignored
    assert np.isnan(S_or).any() and np.isfinite(S_or).any()


def test_sgm_oracle_threads_bit_identical(oracle):
    cv, img = _case(11, 30, 41, 64)
    pen = oracle.sgm_penalties(img)
    n = oracle.get_threads()
    try:
        oracle.set_threads(1)
        a = oracle.sgm_8path(cv, pen)
        oracle.set_threads(4)
        b = oracle.sgm_8path(cv, pen)
    finally:
        oracle.set_threads(n)
    assert a.tobytes() == b.tobytes()


def test_sgm_wraps_diagonals(oracle):
    """Wide-short and tall-narrow images: diagonal paths wrap and restart (:570-572, :702-704)."""
    for (H, W) in [(9, 3), (3, 9)]:
        cv, img = _case(H * W, H, W, 8, invalid_frac=0.0)
        pen = oracle.sgm_penalties(img)
        assert oracle.sgm_8path(cv, pen).tobytes() == sgm_8path_literal(cv, pen).tobytes()


def test_sgm_wta_rule(oracle):
    rng = np.random.default_rng(2)
    S = rng.integers(0, 5, (4, 5, 9)).astype(np.float32)
    d = oracle.wta_sgm(S)
    assert np.array_equal(d, np.argmin(S, axis=-1).astype(np.float32))


def test_post_processing_oracle_properties(oracle):
    rng = np.random.default_rng(4)
    H, W = 9, 12
    dl = rng.integers(0, 6, (H, W)).astype(np.float32)
    dr = rng.integers(0, 6, (H, W)).astype(np.float32)
    a, b = oracle.lr_check(dl, dr)
    for y in range(H):
        for x in range(W):
            if x - dl[y, x] >= 0:
                exp = abs(dl[y, x] - dr[y, int(x - dl[y, x])]) > 1
                assert a[y, x] == exp
            else:
                assert a[y, x] == 0
    filled = oracle.lrc_fill(dl, a)
    assert np.array_equal(filled[a == 0], dl[a == 0])
    med = oracle.median5(filled, dl)
    assert np.array_equal(med[:2], dl[:2]) and np.array_equal(med[:, -2:], dl[:, -2:])
    for y in range(2, H - 2):
        for x in range(2, W - 2):
            assert med[y, x] == np.sort(filled[y - 2:y + 3, x - 2:x + 3].ravel())[12]
