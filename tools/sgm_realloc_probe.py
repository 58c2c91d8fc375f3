"""Placement retries: sets of the four SGM volumes allocated one after another (the previous set kept while the
next is allocated, then freed, empty_cache), each timed with the 7-launch SGM pair (median of 5).  Do fresh
allocations after frees land on fast placements (tools/sgm_block_probe.py: bimodal 5.3 / 5.8 ms)?"""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import _lib, ops  # noqa: E402

H, W, D = 1024, 1024, 192
g = torch.Generator(device="cuda").manual_seed(0)
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
lib = _lib.lib
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p


def med(fn, n=3):
    fn()
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def pair_time(v):
    cl, sl, cr, sr = [t.data_ptr() for t in v]

    def run():
        assert lib.sde_sgm_8path_wta_pair(P(cl), P(pen[0].data_ptr()), P(sl), P(disp[0].data_ptr()), P(cr),
                                          P(pen[1].data_ptr()), P(sr), P(disp[1].data_ptr()), H, W, D, 2, P(s)) == 0
    return med(run)


prev = None
for k in range(10):
    cur = [torch.zeros((H, W, D), device="cuda") for _ in range(4)]
    print(f"set {k}: {pair_time(cur):7.3f} ms   (first VA {cur[0].data_ptr():#x})", flush=True)
    del prev
    torch.cuda.empty_cache()
    prev = cur
