"""Per-phase cycles of the tower's layer-3 launch from a probe build with H16_DIAG & 16384 (tools/variants/tower_h16_diag.h):
every wave's lane 0 sums s_memtime deltas -- MFMA waves: c-block MFMAs, epilogue, barrier wait; stager waves: work,
barrier wait -- and writes them to out[32 block + 4 wave ..].  Printed: median over workgroups per wave role, in
kcycles per launch, and the MFMA floor (1728 MFMAs x 16 cycles per tile).
usage: python tools/tower_phase.py LIB.so [LIB2.so ...]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import mc_cnn, ops  # noqa: E402

H = W = 1024
L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
hin, win = H + 6, W + 6
x = torch.rand((hin, win, 64), device="cuda")
y = torch.empty((hin - 2, win - 2, 64), device="cuda")
words = torch.ones(2, device="cuda")
P, I = ctypes.c_void_p, ctypes.c_int
s = torch.cuda.current_stream().cuda_stream
for so in sys.argv[1:]:
    lib = ctypes.CDLL(so)
    fn = lib.sde_tower_layer_scaled
    fn.argtypes = [P, I, I, P, I, I, I, P, I, P, P, P, P, P, P]
    for _ in range(200):
        rc = fn(x.data_ptr(), hin, win, packed.data_ptr(), L, 64, 3, y.data_ptr(), 8 | 2 | 4, None, None, None,
                words.data_ptr(), words.data_ptr() + 4, s)
        assert rc == 0, rc
    torch.cuda.synchronize()
    st = y.view(-1)[:256 * 32].view(256, 8, 4).double().cpu() / 1e3
    tiles = ((hin - 2 + 15) // 16) * ((win - 2 + 31) // 32) / 256
    print(f"{os.path.basename(so)}: {tiles:.2f} tiles per workgroup, MFMA floor {tiles * 1728 * 16 / 1e3:.0f} kcycles")
    for w in range(8):
        med = [statistics.median(st[:, w, k].tolist()) for k in range(4)]
        role = "mfma " if w < 4 else "stage"
        names = ("cblock", "epilogue", "barrier") if w < 4 else ("work", "barrier", "-")
        print(f"  wave {w} {role}: " + "  ".join(f"{n} {v:7.1f}" for n, v in zip(names, med)))
