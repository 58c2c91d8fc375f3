"""A/B timing of the certified fused CV+WTA (sde_cv_wta, disp only, 1024^2 x 192) in the in-tree
library vs tools/_var/libsde_*.so: round-robin, median of 5 rounds of 5 launches; disparities
and fix-up counts checked identical to the in-tree library's."""
import ctypes
import glob
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib  # noqa: E402
from scenedepthestimation_amd.synthetic import features  # noqa: E402

H, W, D = 1024, 1024, 192
fl = torch.from_numpy(features(H, W, seed=0)).cuda()
fr = torch.from_numpy(features(H, W, seed=1)).cuda()
P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
here = os.path.dirname(os.path.abspath(__file__))
libs = []
for so in [_lib.LIB] + sorted(glob.glob(os.path.join(here, "_var", "libsde_*.so"))):
    lib = ctypes.CDLL(so)
    lib.sde_cv_wta.argtypes = [P, P, I, I, I, I, I, P, P, P, I, P, L, P]
    lib.sde_cv_wta_workspace_bytes.restype = L
    libs.append((os.path.basename(so), lib))
wsb = libs[0][1].sde_cv_wta_workspace_bytes(H, W)
ws = torch.zeros(wsb, dtype=torch.uint8, device="cuda")
disp = torch.empty((H, W), device="cuda")
s = torch.cuda.current_stream().cuda_stream


def run(lib):
    assert lib.sde_cv_wta(fl.data_ptr(), fr.data_ptr(), H, W, 64, 0, D, disp.data_ptr(), None, None, 1,
                          ws.data_ptr(), wsb, s) == 0


ref = None
for name, lib in libs:
    run(lib)
    torch.cuda.synchronize()
    o = (disp.clone(), int(ws[:4].view(torch.int32).item()))
    if ref is None:
        ref = o
    print(f"cv: {name} disparities identical: {torch.equal(o[0], ref[0])}, fix-ups {o[1]}", flush=True)
times = {n: [] for n, _ in libs}
for rnd in range(int(os.environ.get('CV_ROUNDS', '5'))):
    for name, lib in libs:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            run(lib)
        e1.record()
        torch.cuda.synchronize()
        times[name].append(e0.elapsed_time(e1) / 5)
for name, t in times.items():
    print(f"cv  {name:22s} median {statistics.median(t):7.3f} ms  min {min(t):7.3f}  ({' '.join(f'{x:.3f}' for x in t)})",
          flush=True)
