"""Phase breakdown of the certified CV+WTA's compute waves (timing-only build: tools/_var/libsde_cvdiag.so,
SRC=tools/variants/cv_row_diag.hip bash tools/build_file_variant.sh cv_row.hip cvdiag -DCV_DIAG=1).  Wave 0 of each workgroup sums s_memtime
deltas per superstrip phase: 0 = left split (+ next left load issue), 1 = tile sweep (MFMAs + scores),
2 = merges, 3 = the superstrip barrier, 4 = epilogue stores; plus the whole loop in s_memtime and in
s_memrealtime (100 MHz) ticks.  Printed: median over workgroups, cycles per superstrip, and the clock.
usage: python tools/cv_diag.py [H W]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import stereo_pair  # noqa: E402
from scenedepthestimation_amd import _lib, ops  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402

H, W = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1024, 1024)
D = 192
left, right, _ = stereo_pair(H, W, D, seed=0)
m = StereoMatcher(H, W, D)
m.load_images(left, right)
fl, fr = m.features()
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_var", os.environ.get("CV_DIAG_LIB", "libsde_cvdiag.so")))
P, I, L = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
lib.sde_cv_wta.argtypes = [P, P, I, I, I, I, I, P, P, P, I, P, L, P]
disp = torch.empty((H, W), device="cuda")
ws = torch.empty(ops.cv_wta_workspace_bytes(H, W), dtype=torch.uint8, device="cuda")
for rep in range(20):
    rc = lib.sde_cv_wta(fl.data_ptr(), fr.data_ptr(), H, W, 64, 0, D, disp.data_ptr(), None, None,
                        _lib.SDE_CV_CERTIFIED, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0, rc
torch.cuda.synchronize()
st = disp.view(-1)[: 8 * H].view(H, 8).cpu().numpy()
nss = st[0, 7]
names = ["left split", "tile sweep", "merges", "barrier", "epilogue"]
tot = statistics.median(st[:, 5]) / nss
for i, nm in enumerate(names):
    v = statistics.median(st[:, i]) / nss
    print(f"{nm:12s} {v:9.0f} cycles/superstrip  ({100 * v / tot:5.1f} %)")
print(f"{'loop':12s} {tot:9.0f} cycles/superstrip; clock {statistics.median(st[:, 5] / st[:, 6]) / 10:.3f} GHz "
      f"(s_memtime / s_memrealtime x 100 MHz); fix-ups n/a in this build")
