"""How much of the certified CV+WTA's time is per row rather than per pixel?  cv_wta_row2_kernel runs one
workgroup per row (4 rows per CU at 1024 rows): each row starts with a prologue (window 0 loaded and split
before the first superstrip) and ends with its last superstrip's epilogue.  Same pixel count, different
aspect: T(H, W) ~ (H / 256) (c_row + W p), so T(1024, 1024) - T(512, 2048) ~ 2 c_row.
usage: python tools/cv_shape_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import stereo_pair  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402

D = 192


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


shapes = [(1024, 1024), (512, 2048), (256, 4096), (2048, 512), (1024, 512), (512, 1024), (256, 1024)]
ms = {}
for H, W in shapes:
    left, right, _ = stereo_pair(H, W, D, seed=0)
    m = StereoMatcher(H, W, D)
    m.load_images(left, right)
    m.features()
    ms[(H, W)] = m
res = {}
for rnd in range(3):
    for s, m in ms.items():
        res.setdefault(s, []).append(timed(m.cost_wta))
for (H, W), v in res.items():
    fix = int(ms[(H, W)].cv_ws[:4].view(torch.int32).item())
    print(f"H={H:5d} W={W:5d}  rows/CU {H / 256:5.2f}  {statistics.median(v):8.1f} us  "
          f"({' '.join(f'{t:.1f}' for t in v)})  fix-ups {fix}", flush=True)
