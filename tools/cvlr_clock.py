"""Shader clock inside cvlr_dma_kernel: tools/_var/libsde_clk*.so built with CD_SKIP & 128 write
per-workgroup s_memtime / s_memrealtime (100 MHz) deltas into L[0..2*nblocks); median GHz."""
import ctypes
import glob
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd.synthetic import features  # noqa: E402

H, W, D = 1024, 1024, 192
fl = torch.from_numpy(features(H, W, seed=0)).cuda()
fr = torch.from_numpy(features(H, W, seed=1)).cuda()
L = torch.empty((H, W, D), device="cuda")
R = torch.empty((H, W, D), device="cuda")
P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
nb = H * ((D + 63) // 64)
for so in sorted(glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_var", "libsde_clk*.so"))):
    lib = ctypes.CDLL(so)
    lib.sde_cost_volume.argtypes = [P, P, I, I, I, I, I, I, F, P, P, P]
    s = torch.cuda.current_stream().cuda_stream
    for _ in range(6):
        assert lib.sde_cost_volume(fl.data_ptr(), fr.data_ptr(), H, W, 64, D, 1, 3, 1.0, L.data_ptr(), R.data_ptr(), s) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    assert lib.sde_cost_volume(fl.data_ptr(), fr.data_ptr(), H, W, 64, D, 1, 3, 1.0, L.data_ptr(), R.data_ptr(), s) == 0
    e1.record()
    torch.cuda.synchronize()
    v = L.view(-1)[: 2 * nb].view(nb, 2).double().cpu()
    ok = v[:, 1] > 0
    ghz = (v[ok, 0] / (v[ok, 1] / 100e6) / 1e9)
    print(f"{os.path.basename(so):22s} {e0.elapsed_time(e1):.3f} ms  clock median {ghz.median():.3f} GHz "
          f"(p10 {ghz.quantile(0.1):.3f}, p90 {ghz.quantile(0.9):.3f})", flush=True)
