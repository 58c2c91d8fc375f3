"""Placement sensitivity of the 7-launch SGM pair (1024^2 x 192) for the library and each tools/_var/libsde_sgm*.so
probe build (e.g. SGM_SKEW: line streams started out of lock step, tools/variants/sgm_probe.hip): for every library,
NSETS sets of the four volumes allocated one after another (the previous set held while the next is allocated --
the allocation pattern that lands sets on different physical memory), each timed (median of 3).
Prints every set's time and the median / min / max per library; disparities checked identical to the library's.
usage: python tools/sgm_skew_probe.py [NSETS]"""
import ctypes
import glob
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib, ops  # noqa: E402

NSETS = int(sys.argv[1]) if len(sys.argv) > 1 else 8
H, W, D = 1024, 1024, 192
g = torch.Generator(device="cuda").manual_seed(0)
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p
here = os.path.dirname(os.path.abspath(__file__))
libs = [("libsde.so", _lib.lib)] + [(os.path.basename(p), ctypes.CDLL(p))
                                    for p in sorted(glob.glob(os.path.join(here, "_var", "libsde_sgm*.so")))]


def pair_time(lib, v):
    cl, sl, cr, sr = [t.data_ptr() for t in v]

    def run():
        assert lib.sde_sgm_8path_wta_pair(P(cl), P(pen[0].data_ptr()), P(sl), P(disp[0].data_ptr()), P(cr),
                                          P(pen[1].data_ptr()), P(sr), P(disp[1].data_ptr()), H, W, D, 2, P(s)) == 0
    run()
    ts = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


costs = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
ref = None
for name, lib in libs:
    prev, ts = None, []
    for k in range(NSETS):
        cur = [costs[0].clone(), torch.empty((H, W, D), device="cuda"), costs[1].clone(), torch.empty((H, W, D), device="cuda")]
        ts.append(pair_time(lib, cur))
        if k == 0:
            d = torch.cat([disp[0].flatten(), disp[1].flatten()]).clone()
            if ref is None:
                ref = d
            same = bool(torch.equal(d, ref))
        del prev
        torch.cuda.empty_cache()
        prev = cur
    del prev
    torch.cuda.empty_cache()
    print(f"{name:24s} sets: {' '.join(f'{t:.3f}' for t in ts)}  median {statistics.median(ts):.3f} min {min(ts):.3f} "
          f"max {max(ts):.3f} ms  disparities identical: {same}", flush=True)
