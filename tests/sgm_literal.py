"""Literal pure-Python restatement of the reference's Numba SGM kernels (test-only).

Follows process_functional.py:265-797 statement by statement: a "warp" of D/4
lanes holding 4 disparities each, the shfl_up/shfl_down neighbour exchange, the
is_first / is_copy / is_cal_min flags and the per-kernel traversal (first step,
``for i in range(1, max_iter - 1)`` loop, final step without the min).  Python
floats are float64, matching Numba's unified loop-carried types.  Slow: small
images only.  Used to cross-check the C oracle's restructured restatement.
"""
import numpy as np


def _interation(row, col, P1, P2, old, min_cost, min_cost_P2, is_copy, is_first, is_cal_min, cv, S):
    """min_cost / min_cost_P2: one value per lane (the reference's registers are per thread)."""
    nl = cv.shape[2] // 4
    c = [[float(cv[row, col, 4 * l + i]) for i in range(4)] for l in range(nl)]   # c1..c4 per lane
    if not (is_first or is_copy):
        for l in range(nl):
            o1, o2, o3, o4 = old[l]
            pre = old[l - 1][3] if l > 0 else o4         # shfl_up(old_values4, 1)
            nxt = old[l + 1][0] if l < nl - 1 else o1    # shfl_down(old_values1, 1)
            if l == 0:                                   # disp // 4 == 0
                pre = o1
            if l == nl - 1:                              # disp // 4 == last lane
                nxt = o4
            mc, mcp2 = min_cost[l], min_cost_P2[l]
            c[l][0] += min(min(pre + P1, o1), min(o2 + P1, mcp2)) - mc
            c[l][1] += min(min(o1 + P1, o2), min(o3 + P1, mcp2)) - mc
            c[l][2] += min(min(o2 + P1, o3), min(o4 + P1, mcp2)) - mc
            c[l][3] += min(min(o3 + P1, o4), min(nxt + P1, mcp2)) - mc
    for l in range(nl):
        for i in range(4):
            S[row, col, 4 * l + i] = np.float32(float(S[row, col, 4 * l + i]) + c[l][i])
    if is_cal_min:
        # m1 = min(c1, c2); m2 = min(c3, c4); min_cost = min(m1, m2); then
        # min_cost = min(min_cost, shfl_xor_sync(min_cost, k)) for k = 1, 2, 4, 8, 16 (one 32-lane warp)
        # (D != 128: the build's generalisation -- lanes padded to a power of two with +inf)
        nlp = 1
        while nlp < nl:
            nlp <<= 1
        m = [min(min(v[0], v[1]), min(v[2], v[3])) for v in c] + [float("inf")] * (nlp - nl)
        k = 1
        while k < nlp:
            m = [min(m[l], m[l ^ k]) for l in range(nlp)]
            k <<= 1
        m = m[:nl]
        min_cost = m
        min_cost_P2 = [v + P2 for v in m]
    return c, min_cost, min_cost_P2


def _pen(p, r, c, ch):
    return float(p[r, c, ch])


def _run_line(steps, cv, S):
    """steps: list of (row, col, P1, P2, is_copy, is_first, is_cal_min)."""
    nl = cv.shape[2] // 4
    old = [[1.0] * 4 for _ in range(nl)]
    mc, mcp2 = [1.0] * nl, [1.0] * nl
    for (r, c, P1, P2, cp, first, calmin) in steps:
        old, mc, mcp2 = _interation(r, c, P1, P2, old, mc, mcp2, cp, first, calmin, cv, S)


def vertical(cv, pen, S, down):
    rows, cols = cv.shape[:2]
    ch1, ch2 = (2, 3) if down else (0, 1)
    step = 1 if down else -1
    for col in range(cols):
        row = 0 if down else rows - 1
        max_iter = rows - 1
        steps = []
        prev_ok = (row - 1 >= 0) if down else (row + 1 < rows)
        P1 = _pen(pen, row - step, col, ch1) if prev_ok else 0
        steps.append((row, col, P1, _pen(pen, row, col, ch2), False, True, True))
        for _ in range(1, max_iter - 1):
            row += step
            steps.append((row, col, _pen(pen, row - step, col, ch1), _pen(pen, row, col, ch2), False, False, True))
        row += step
        steps.append((row, col, _pen(pen, row - step, col, ch1), _pen(pen, row, col, ch2), False, False, False))
        _run_line(steps, cv, S)


def horizontal(cv, pen, S, right):
    rows, cols = cv.shape[:2]
    ch1, ch2 = (6, 7) if right else (4, 5)
    step = 1 if right else -1
    for row in range(rows):
        col = 0 if right else cols - 1
        max_iter = cols - 1
        steps = []
        prev_ok = (col - 1 >= 0) if right else (col + 1 < cols)
        P1 = _pen(pen, row, col - step, ch1) if prev_ok else 0
        steps.append((row, col, P1, _pen(pen, row, col, ch2), False, True, True))
        for _ in range(1, max_iter - 1):
            col += step
            steps.append((row, col, _pen(pen, row, col - step, ch1), _pen(pen, row, col, ch2), False, False, True))
        col += step
        steps.append((row, col, _pen(pen, row, col - step, ch1), _pen(pen, row, col, ch2), False, False, False))
        _run_line(steps, cv, S)


def diagonal(cv, pen, S, down, right):
    rows, cols = cv.shape[:2]
    ch1 = {(True, True): 10, (False, True): 12, (True, False): 8, (False, False): 14}[(down, right)]
    ch2 = ch1 + 1
    dr = 1 if down else -1
    dc = 1 if right else -1

    def p1(row, col):
        pr, pc = row - dr, col - dc
        if (pc < 0 if right else pc >= cols) or (pr < 0 if down else pr >= rows):
            return 0
        return _pen(pen, pr, pc, ch1)

    def advance(row, col):
        row += dr
        col += dc
        cp = False
        if right and col >= cols:
            col, cp = 0, True
        if not right and col < 0:
            col, cp = cols - 1, True
        return row, col, cp

    for start in range(cols):
        row = 0 if down else rows - 1
        col = start
        max_iter = rows - 1
        steps = [(row, col, p1(row, col), _pen(pen, row, col, ch2), False, True, True)]
        for _ in range(1, max_iter - 1):
            row, col, cp = advance(row, col)
            steps.append((row, col, p1(row, col), _pen(pen, row, col, ch2), cp, False, True))
        row, col, cp = advance(row, col)
        steps.append((row, col, p1(row, col), _pen(pen, row, col, ch2), cp, False, False))
        _run_line(steps, cv, S)


def sgm_8path_literal(cv, pen):
    """One side (k loop body) of the 8 launches, process_functional.py:1166-1203."""
    assert cv.shape[2] % 4 == 0
    S = np.zeros(cv.shape, np.float32)
    vertical(cv, pen, S, True)
    vertical(cv, pen, S, False)
    horizontal(cv, pen, S, True)
    horizontal(cv, pen, S, False)
    diagonal(cv, pen, S, True, True)
    diagonal(cv, pen, S, False, True)
    diagonal(cv, pen, S, True, False)
    diagonal(cv, pen, S, False, False)
    return S
