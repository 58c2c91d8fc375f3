"""Does the SGM pair's time depend on where its volumes sit in HBM?  The four [H][W][D] volumes
(cost L/R, S L/R) are carved out of one allocation at chosen byte offsets and the 7-launch pair
(sde_sgm_8path_wta_pair) is timed per layout, round-robin, median of 5; disparities checked
identical across layouts.  usage: python tools/sgm_offsets.py"""
import ctypes
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib, ops  # noqa: E402

H, W, D = 1024, 1024, 192
V = H * W * D * 4
KB, MB = 1024, 1024 * 1024
# name -> byte offsets of (cv_l, S_l, cv_r, S_r) inside the buffer; the volumes sit 4 MB apart
# (plus the layout's shift), so no shift makes two of them overlap
G = 4 * MB
layouts = {
    "packed":        (0, V + G, 2 * V + 2 * G, 3 * V + 3 * G),
    "S+4K":          (0, V + G + 4 * KB, 2 * V + 2 * G, 3 * V + 3 * G + 4 * KB),
    "S+64K":         (0, V + G + 64 * KB, 2 * V + 2 * G, 3 * V + 3 * G + 64 * KB),
    "S+1M":          (0, V + G + 1 * MB, 2 * V + 2 * G, 3 * V + 3 * G + 1 * MB),
    "S+3M+8K":       (0, V + G + 3 * MB + 8 * KB, 2 * V + 2 * G, 3 * V + 3 * G + 3 * MB + 8 * KB),
    "R+2K":          (0, V + G, 2 * V + 2 * G + 2 * KB, 3 * V + 3 * G + 2 * KB),
    "R+256K,S+12K":  (0, V + G + 12 * KB, 2 * V + 2 * G + 256 * KB, 3 * V + 3 * G + 268 * KB),
}
buf = torch.empty(4 * V + 4 * G, dtype=torch.uint8, device="cuda")
base = buf.data_ptr()
g = torch.Generator(device="cuda").manual_seed(0)
src = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
lib = _lib.lib
s = torch.cuda.current_stream().cuda_stream


def place(off):
    o = off[:]
    for k, c in ((0, 0), (2, 1)):   # copy the costs into place
        dst = torch.as_strided(buf[o[k]:o[k] + V].view(torch.float32), (H, W, D), (W * D, D, 1))
        dst.copy_(src[c])


def run(off):
    assert lib.sde_sgm_8path_wta_pair(ctypes.c_void_p(base + off[0]), ctypes.c_void_p(pen[0].data_ptr()),
                                      ctypes.c_void_p(base + off[1]), ctypes.c_void_p(disp[0].data_ptr()),
                                      ctypes.c_void_p(base + off[2]), ctypes.c_void_p(pen[1].data_ptr()),
                                      ctypes.c_void_p(base + off[3]), ctypes.c_void_p(disp[1].data_ptr()),
                                      H, W, D, 2, ctypes.c_void_p(s)) == 0


ref = None
times = {n: [] for n in layouts}
for rnd in range(5):
    for name, off in layouts.items():
        place(list(off))
        run(off)
        if rnd == 0:
            torch.cuda.synchronize()
            out = torch.cat([d.flatten() for d in disp]).clone()
            ref = out if ref is None else ref
            print(f"{name}: disparities identical to the first layout's: {torch.equal(out, ref)}", flush=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run(off)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 3)
print(f"buffer base 0x{base:x}")
for name, t in times.items():
    print(f"{name:14s} median {statistics.median(t):7.3f} ms  ({' '.join(f'{x:.3f}' for x in t)})", flush=True)
