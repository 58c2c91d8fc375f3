"""A/B of the certified CV+WTA (sde_cv_wta, mode certified) across tools/_var/libsde_*.so and the library
itself: real tower features of a synthetic pair per shape, round-robin over the libraries, 3 rounds, median.
Every library's disparity map, argmin and min cost must equal the library's own (bit for bit).
usage: python tools/cv_variants.py [H W ...]"""
import ctypes
import glob
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import stereo_pair  # noqa: E402
from scenedepthestimation_amd import _lib, ops  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402

D = 192
a = [int(v) for v in sys.argv[1:]]
shapes = list(zip(a[::2], a[1::2])) or [(1024, 1024), (375, 450), (512, 2048), (257, 1000)]
P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
here = os.path.dirname(os.path.abspath(__file__))
libs = []
for so in [_lib.LIB] + sorted(glob.glob(os.path.join(here, "_var", "libsde_*.so"))):
    lib = ctypes.CDLL(so)
    lib.sde_cv_wta.argtypes = [P, P, I, I, I, I, I, P, P, P, I, P, L, P]
    libs.append((os.path.basename(so), lib))


def timed(fn, n=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


cases = []
for H, W in shapes:
    left, right, _ = stereo_pair(H, W, D, seed=0)
    m = StereoMatcher(H, W, D)
    m.load_images(left, right)
    fl, fr = m.features()
    outs = {}
    for name, lib in libs:
        disp = torch.empty((H, W), device="cuda")
        mc = torch.empty((H, W), device="cuda")
        am = torch.empty((H, W), dtype=torch.int32, device="cuda")
        ws = torch.empty(ops.cv_wta_workspace_bytes(H, W), dtype=torch.uint8, device="cuda")

        def run(lib=lib, disp=disp, mc=mc, am=am, ws=ws, H=H, W=W, fl=fl, fr=fr, want_min=True):
            s = torch.cuda.current_stream().cuda_stream
            rc = lib.sde_cv_wta(fl.data_ptr(), fr.data_ptr(), H, W, 64, 0, D, disp.data_ptr(),
                                mc.data_ptr() if want_min else None, am.data_ptr() if want_min else None,
                                _lib.SDE_CV_CERTIFIED, ws.data_ptr(), ws.numel(), s)
            assert rc == 0, rc
        run()
        torch.cuda.synchronize()
        outs[name] = (disp.clone(), mc.clone(), am.clone(), int(ws[:4].view(torch.int32).item()))
        cases.append(((H, W), name, lambda run=run: run(want_min=False)))
    ref = outs[libs[0][0]]
    for name, o in outs.items():
        same = torch.equal(o[0], ref[0]) and torch.equal(o[2], ref[2]) and \
            torch.equal(o[1].view(torch.int32), ref[1].view(torch.int32))
        print(f"{H}x{W} {name:24s} identical to {libs[0][0]}: {same}  fix-ups {o[3]}", flush=True)
res = {}
for rnd in range(3):
    for shape, name, fn in cases:
        res.setdefault((shape, name), []).append(timed(fn))
for (shape, name), v in res.items():
    print(f"{shape[0]:5d}x{shape[1]:<5d} {name:24s} {statistics.median(v):8.1f} us  ({' '.join(f'{t:.1f}' for t in v)})",
          flush=True)
