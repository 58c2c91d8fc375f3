"""Time sde_sgm_8path_wta_pair (both sides, 7 launches) of each tools/_var/libsde_sgm_<name>.so at
H x W x D, interleaved over rounds; check every variant's S and disparity maps bit-identical to the
first's."""
import ctypes
import glob
import os
import sys

import torch

H, W, D = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1024, 1024, 192)))
g = torch.Generator(device="cuda").manual_seed(0)
cv = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
S = [torch.empty((H, W, D), device="cuda") for _ in range(2)]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
pen = [torch.empty((H, W, 16), device="cuda") for _ in range(2)]
P, I = ctypes.c_void_p, ctypes.c_int
libs = []
for so in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_var", "libsde_sgm_*.so"))):
    lib = ctypes.CDLL(so)
    lib.sde_sgm_penalties.argtypes = [P, I, I, ctypes.c_double, ctypes.c_double, ctypes.c_int64, ctypes.c_double,
                                      P, P]
    lib.sde_sgm_8path_wta_pair.argtypes = [P] * 8 + [I, I, I, I, P]
    libs.append((os.path.basename(so), lib))
s = torch.cuda.current_stream().cuda_stream
for k in range(2):
    assert libs[0][1].sde_sgm_penalties(img[k].data_ptr(), H, W, 0.1, 0.5, 10, 2.0, pen[k].data_ptr(), s) == 0


def run(lib):
    assert lib.sde_sgm_8path_wta_pair(cv[0].data_ptr(), pen[0].data_ptr(), S[0].data_ptr(), disp[0].data_ptr(),
                                      cv[1].data_ptr(), pen[1].data_ptr(), S[1].data_ptr(), disp[1].data_ptr(),
                                      H, W, D, 2, s) == 0     # SDE_SGM_ZERO_DU_PENALTIES


ref = None
times = {n: [] for n, _ in libs}
for rnd in range(5):
    for n, lib in libs:
        run(lib)
        if rnd == 0:
            out = torch.cat([t.flatten() for t in (disp[0], disp[1], S[0], S[1])]).view(torch.int32).clone()
            ref = out if ref is None else ref
            print(f"{n}: S + disparities bit-identical to {libs[0][0]}: {torch.equal(out, ref)}", flush=True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            run(lib)
        e1.record()
        torch.cuda.synchronize()
        times[n].append(e0.elapsed_time(e1) / 3)
for n, t in times.items():
    print(f"{n:22s} " + " ".join(f"{x:.3f}" for x in t) + f"  median {sorted(t)[len(t) // 2]:.3f} ms", flush=True)
