"""One middle tower layer (layer 3, c-block layouts) at 1024^2, `reps` launches, with the library
or a tools/_var variant (argv: [so path] [precision] [reps]) -- for rocprofv3 PMC passes."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib, mc_cnn, ops  # noqa: E402

so = sys.argv[1] if len(sys.argv) > 1 and sys.argv[1] != "lib" else _lib.LIB
prec = sys.argv[2] if len(sys.argv) > 2 else "f16x3"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
H = W = 1024
L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
hin, win = H + 6, W + 6
x = torch.rand((hin, win, 64), device="cuda")
y = torch.empty((hin - 2, win - 2, 64), device="cuda")
words = torch.ones(2, device="cuda")
P, I = ctypes.c_void_p, ctypes.c_int
lib = ctypes.CDLL(so)
fn = lib.sde_tower_layer_scaled
fn.argtypes = [P, I, I, P, I, I, I, P, I, P, P, P, P, P, P]
flag = {"bf16x6": 1, "f16x3": 8}[prec]
s = torch.cuda.current_stream().cuda_stream
for _ in range(reps):
    rc = fn(x.data_ptr(), hin, win, packed.data_ptr(), L, 64, 3, y.data_ptr(), flag | 2 | 4, None, None, None,
            words.data_ptr(), words.data_ptr() + 4, s)
    assert rc == 0, rc
torch.cuda.synchronize()
