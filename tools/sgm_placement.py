"""Does the SGM pair's time depend on which HBM pages its volumes land on?  NSET separate sets of
four [H][W][D] volumes (cost L/R, S L/R), each its own allocation, hold the same costs; the 7-launch
pair (sde_sgm_8path_wta_pair) runs on each set in turn (run under rocprofv3 --kernel-trace for the
per-direction split).  Same disparities for every set.  With "contig", the odd sets are allocated
by hipExtMallocWithFlags(hipDeviceMallocContiguous) instead of the torch allocator.
usage: python tools/sgm_placement.py [NSET] [contig]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib, ops  # noqa: E402

H, W, D = 1024, 1024, 192
NSET = int(sys.argv[1]) if len(sys.argv) > 1 else 5
g = torch.Generator(device="cuda").manual_seed(0)
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
CONTIG = len(sys.argv) > 2 and sys.argv[2] == "contig"
hip = ctypes.CDLL("libamdhip64.so")
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
keep = []


class Raw:
    """a device buffer from hipExtMallocWithFlags, viewed as an [H][W][D] float32 tensor"""
    def __init__(self, flags):
        p = ctypes.c_void_p()
        assert hip.hipExtMallocWithFlags(ctypes.byref(p), H * W * D * 4, flags) == 0
        self.p = p.value
        keep.append(self)

    def data_ptr(self):
        return self.p

    def copy_(self, t):
        assert hip.hipMemcpy(ctypes.c_void_p(self.p), ctypes.c_void_p(t.data_ptr()), ctypes.c_size_t(H * W * D * 4),
                             3) == 0   # device to device


def vol(k):
    return Raw(0x4) if CONTIG and k % 2 == 1 else torch.empty((H, W, D), device="cuda")


sets = []
for k in range(NSET):
    cv = [vol(k) for _ in range(2)]
    S = [vol(k) for _ in range(2)]
    g2 = torch.Generator(device="cuda").manual_seed(1)
    for c in cv:
        c.copy_(torch.rand((H, W, D), device="cuda", generator=g2))
    sets.append((cv, S))
lib = _lib.lib
s = torch.cuda.current_stream().cuda_stream


def run(cv, S):
    P = ctypes.c_void_p
    assert lib.sde_sgm_8path_wta_pair(P(cv[0].data_ptr()), P(pen[0].data_ptr()), P(S[0].data_ptr()),
                                      P(disp[0].data_ptr()), P(cv[1].data_ptr()), P(pen[1].data_ptr()),
                                      P(S[1].data_ptr()), P(disp[1].data_ptr()), H, W, D, 2, P(s)) == 0


ref = None
times = [[] for _ in sets]
for rnd in range(4):
    for k, (cv, S) in enumerate(sets):
        run(cv, S)
        if rnd == 0:
            torch.cuda.synchronize()
            out = torch.cat([d.flatten() for d in disp]).clone()
            ref = out if ref is None else ref
            print(f"set {k}: cv 0x{cv[0].data_ptr():x} 0x{cv[1].data_ptr():x} S 0x{S[0].data_ptr():x} "
                  f"0x{S[1].data_ptr():x}; disparities identical to set 0's: {torch.equal(out, ref)}", flush=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(2):
            run(cv, S)
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 2)
for k, t in enumerate(times):
    print(f"set {k} median {statistics.median(t):7.3f} ms  ({' '.join(f'{x:.3f}' for x in t)})", flush=True)
