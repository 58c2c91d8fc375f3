"""Time one middle tower layer (layer 3, c-block layouts) of each tools/_var/libsde_t<bits>.so
(see tower_variants.sh) and of the library itself, for bf16x6 and f16x3."""
import ctypes
import glob
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import mc_cnn, ops  # noqa: E402

H = W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
hin, win = H + 6, W + 6
x = torch.rand((hin, win, 64), device="cuda")
y = torch.empty((hin - 2, win - 2, 64), device="cuda")
words = torch.ones(2, device="cuda")
P, I = ctypes.c_void_p, ctypes.c_int
here = os.path.dirname(os.path.abspath(__file__))
sos = sorted(glob.glob(os.path.join(here, "_var", "libsde_*.so")))
from scenedepthestimation_amd import _lib  # noqa: E402
for so in [_lib.LIB] + sos:
    lib = ctypes.CDLL(so)
    fn = lib.sde_tower_layer_scaled
    fn.argtypes = [P, I, I, P, I, I, I, P, I, P, P, P, P, P, P]
    s = torch.cuda.current_stream().cuda_stream
    for prec, flag in (("bf16x6", 1), ("f16x3", 8)):
        def run():
            words[1] = 0
            rc = fn(x.data_ptr(), hin, win, packed.data_ptr(), L, 64, 3, y.data_ptr(), flag | 2 | 4, None, None, None,
                    words.data_ptr(), words.data_ptr() + 4, s)
            assert rc == 0, rc
        for _ in range(20):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        msg = ""
        if "clk" in os.path.basename(so):   # TOWER_DIAG & 128: per-workgroup cycle / 100 MHz-tick deltas
            st = y.view(-1)[:512].view(256, 2).double()
            ghz = (st[:, 0] / st[:, 1] * 0.1).median().item()
            msg = f"  in-kernel clock {ghz:.3f} GHz, {st[:, 0].median().item() / 1e3:.0f} kcycles"
        print(f"{os.path.basename(so):20s} {prec:7s} {e0.elapsed_time(e1) / 20 * 1e3:8.1f} us{msg}", flush=True)
