"""Time sde_cost_volume (HWD, L|R) of each tools/_var/libsde_<bits>.so (see cvlr_variants.sh)."""
import ctypes
import glob
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd.synthetic import features  # noqa: E402

H, W, D = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1024, 1024, 192)))
fl = torch.from_numpy(features(H, W, seed=0)).cuda()
fr = torch.from_numpy(features(H, W, seed=1)).cuda()
L = torch.empty((H, W, D), device="cuda")
R = torch.empty((H, W, D), device="cuda")
P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
here = os.path.dirname(os.path.abspath(__file__))
for so in sorted(glob.glob(os.path.join(here, "_var", "libsde_*.so")), key=lambda s: int(s.split("_")[-1][:-3])):
    lib = ctypes.CDLL(so)
    fn = lib.sde_cost_volume
    fn.argtypes = [P, P, I, I, I, I, I, I, F, P, P, P]
    s = torch.cuda.current_stream().cuda_stream

    def run():
        rc = fn(fl.data_ptr(), fr.data_ptr(), H, W, 64, D, 1, 3, 1.0, L.data_ptr(), R.data_ptr(), s)
        assert rc == 0, rc
    for _ in range(3):
        run()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(f"{os.path.basename(so):20s} {e0.elapsed_time(e1) / 10:8.3f} ms", flush=True)
