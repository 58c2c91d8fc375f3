"""Per-buffer or per-combination?  Eight separately allocated [1024][1024][192] volumes; the 7-launch SGM pair timed
(median of 5) with several assignments of four of them to (cost L, S L, cost R, S R), each assignment twice, plus a
streaming read+write of each volume alone (x.mul_(1): ~1.6 GB) -- which volumes make the pair slow?"""
import ctypes
import itertools
import random
import statistics
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import _lib, ops  # noqa: E402

H, W, D = 1024, 1024, 192
g = torch.Generator(device="cuda").manual_seed(0)
vols = [torch.zeros((H, W, D), device="cuda") for _ in range(8)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
lib = _lib.lib
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p


def med(fn, n=5):
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


for i, v in enumerate(vols):
    print(f"vol {i}: stream r+w {med(lambda: v.mul_(1.0)):6.3f} ms", flush=True)
rng = random.Random(1)
combos = [(0, 1, 2, 3), (4, 5, 6, 7)] + [tuple(rng.sample(range(8), 4)) for _ in range(8)]
for rep in range(2):
    for c in combos:
        cl, sl, cr, sr = [vols[k].data_ptr() for k in c]

        def run():
            assert lib.sde_sgm_8path_wta_pair(P(cl), P(pen[0].data_ptr()), P(sl), P(disp[0].data_ptr()), P(cr),
                                              P(pen[1].data_ptr()), P(sr), P(disp[1].data_ptr()), H, W, D, 2,
                                              P(s)) == 0
        print(f"rep {rep} (cL, sL, cR, sR) = {c}: {med(run):7.3f} ms", flush=True)
