"""Generate the golden vectors that pin the CPU oracle (run in the build container only).

The reference module `process_functional.py` cannot be imported here (it imports
tensorflow and numba, both absent: ordinary ModuleNotFoundError, no permission
denial).  Its CPU path, however, is pure NumPy:

  * ``compute_cost_volume``  process_functional.py:48-73
  * ``WTA``                  process_functional.py:76-93
  * ``WTA1``                 process_functional.py:96-113

This script parses the reference source text with ``ast``, compiles exactly those
three function definitions and executes them on seeded inputs.  Only the
inputs/outputs are written (``golden_cpu_path.npz``); no reference source travels.

Usage (in the build container, where /root/reference exists):

    python tests/golden/make_golden.py

The produced fixture is committed; tests never read /root/reference.
"""
from __future__ import annotations

import ast
import os
import sys
import time
from datetime import datetime

import numpy as np

REF = os.environ.get("SDE_REFERENCE_DIR", "/root/reference")
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden_cpu_path.npz")
WANTED = ("compute_cost_volume", "WTA", "WTA1")


def load_reference_cpu_functions():
    src_path = os.path.join(REF, "process_functional.py")
    with open(src_path, "r") as fh:
        tree = ast.parse(fh.read(), filename=src_path)
    defs = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in WANTED]
    found = sorted(n.name for n in defs)
    if found != sorted(WANTED):
        raise RuntimeError(f"expected {WANTED} in {src_path}, found {found}")
    mod = ast.Module(body=defs, type_ignores=[])
    ns = {"np": np, "datetime": datetime, "time": time,
          # the reference functions print progress lines; keep the generator quiet
          "print": lambda *a, **k: None}
    exec(compile(mod, src_path, "exec"), ns)
    return ns["compute_cost_volume"], ns["WTA"], ns["WTA1"]


def l2n(x):
    n = np.sqrt(np.sum(x.astype(np.float64) ** 2, axis=-1, keepdims=True))
    return (x / np.maximum(n, 1e-12)).astype(np.float32)


def make_cases(rng):
    """(name, fl, fr, ndisp) tuples covering the reference's edge cases."""
    cases = []
    # plain L2-normalised features (the tower's output domain), C = 64
    for (h, w, d) in [(6, 20, 8), (5, 40, 16), (4, 70, 64), (3, 9, 12)]:
        fl = l2n(rng.standard_normal((h, w, 64)).astype(np.float32))
        fr = l2n(rng.standard_normal((h, w, 64)).astype(np.float32))
        cases.append((f"rand_h{h}_w{w}_d{d}", fl, fr, d))
    # right = left shifted by a known disparity band (a "matchable" pair)
    h, w, d = 6, 48, 16
    base = l2n(rng.standard_normal((h, w + d, 64)).astype(np.float32))
    fl = base[:, d:].copy()
    shift = 5
    fr = np.concatenate([base[:, d - shift:w + d - shift]], axis=1).copy()
    cases.append(("shifted5_h6_w48_d16", fl, fr, d))
    # all-negative dots: every valid cost > 0, so the -0.0 invalid voxels win the argmin
    h, w, d = 4, 24, 10
    fl = np.abs(l2n(rng.standard_normal((h, w, 64)).astype(np.float32)))
    fr = -np.abs(l2n(rng.standard_normal((h, w, 64)).astype(np.float32)))
    cases.append(("negdot_h4_w24_d10", fl, fr, d))
    # exact ties: constant right features -> equal costs for all valid d (first-min rule)
    h, w, d = 3, 16, 8
    fl = l2n(rng.standard_normal((h, w, 64)).astype(np.float32))
    fr = np.broadcast_to(l2n(rng.standard_normal((1, 1, 64)).astype(np.float32)), (h, w, 64)).copy()
    cases.append(("ties_h3_w16_d8", fl, fr, d))
    # zero / signed-zero features: dot = -0.0 and +0.0 paths through NumPy's 0.0 + sum
    h, w, d = 2, 12, 6
    fl = np.zeros((h, w, 64), np.float32)
    fl[:, ::2] = -0.0
    fr = np.zeros((h, w, 64), np.float32)
    fr[:, 1::3] = -0.0
    fl[1, 5] = l2n(rng.standard_normal((64,)).astype(np.float32))
    cases.append(("zeros_h2_w12_d6", fl, fr, d))
    # un-normalised wide-range features (rounding stress), C = 64
    h, w, d = 4, 30, 12
    fl = (rng.standard_normal((h, w, 64)) * np.exp(rng.uniform(-6, 6, (h, w, 64)))).astype(np.float32)
    fr = (rng.standard_normal((h, w, 64)) * np.exp(rng.uniform(-6, 6, (h, w, 64)))).astype(np.float32)
    cases.append(("wide_h4_w30_d12", fl, fr, d))
    # other channel counts exercise every branch of NumPy's pairwise sum
    for c in (1, 3, 8, 20, 100, 128, 136, 200):
        h, w, d = 3, 14, 7
        fl = (rng.standard_normal((h, w, c)) * 3).astype(np.float32)
        fr = (rng.standard_normal((h, w, c)) * 3).astype(np.float32)
        cases.append((f"chan{c}_h3_w14_d7", fl, fr, d))
    # ndisp > width (whole columns of invalid voxels) and a 1x1 image
    fl = l2n(rng.standard_normal((2, 5, 64)).astype(np.float32))
    fr = l2n(rng.standard_normal((2, 5, 64)).astype(np.float32))
    cases.append(("dgtw_h2_w5_d9", fl, fr, 9))
    fl = l2n(rng.standard_normal((1, 1, 64)).astype(np.float32))
    fr = l2n(rng.standard_normal((1, 1, 64)).astype(np.float32))
    cases.append(("one_h1_w1_d1", fl, fr, 1))
    return cases


def main():
    compute_cost_volume, WTA, WTA1 = load_reference_cpu_functions()
    rng = np.random.default_rng(20261015)
    out = {}
    names = []
    for name, fl, fr, d in make_cases(rng):
        cv = compute_cost_volume(fl, fr, d)            # [D,H,W]
        disp = WTA1(cv)                                 # [H,W] f32
        disp_hwd = WTA(np.ascontiguousarray(np.transpose(cv, (1, 2, 0))))   # [H,W,D] variant
        assert cv.dtype == np.float32 and disp.dtype == np.float32
        assert np.array_equal(disp, disp_hwd)
        out[f"{name}__fl"] = fl
        out[f"{name}__fr"] = fr
        out[f"{name}__ndisp"] = np.int64(d)
        out[f"{name}__cv"] = cv
        out[f"{name}__disp"] = disp
        names.append(name)
    # a WTA-only case with exact ties and -0.0/+0.0 ties in an [H,W,D] volume
    vol = rng.integers(-3, 4, size=(5, 7, 11)).astype(np.float32)
    vol[0, 0, :] = 0.0
    vol[0, 0, 3] = -0.0
    vol[1, 1, :] = np.float32(np.inf)
    vol[1, 1, 9] = np.float32(1e30)
    out["wta_hwd__vol"] = vol
    out["wta_hwd__disp"] = WTA(vol)
    out["wta_dhw__vol"] = np.ascontiguousarray(np.transpose(vol, (2, 0, 1)))
    out["wta_dhw__disp"] = WTA1(out["wta_dhw__vol"])
    out["__cases__"] = np.array(names)
    out["__numpy_version__"] = np.array(np.__version__)
    np.savez_compressed(OUT, **out)
    print(f"wrote {OUT}: {len(names)} cost-volume cases", file=sys.stderr)


if __name__ == "__main__":
    main()
