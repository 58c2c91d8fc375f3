"""Run tools/_var/split_probe.so (tools/probes/split_probe.hip) on 2^26 test values: log-uniform magnitudes
over [2^-40, 2^8] of both signs (every fp16 normal/subnormal regime of x * 2^8), the tower's features at
1024^2, and zeros.  usage: python tools/probes/split_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

here = os.path.dirname(os.path.abspath(__file__))
lib = ctypes.CDLL(os.path.join(here, "..", "_var", "split_probe.so"))
lib.split_probe.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
rng = np.random.default_rng(0)
n = 1 << 26
mag = np.exp2(rng.uniform(-40, 8, n)).astype(np.float32) * rng.choice([-1, 1], n).astype(np.float32)
sets = {"log-uniform 2^-40..2^8": mag, "gaussian 0.1": (rng.standard_normal(n) * 0.1).astype(np.float32)}
sys.path.insert(0, os.path.join(here, "..", ".."))
from bench import stereo_pair  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402
m = StereoMatcher(1024, 1024, 192)
left, right, _ = stereo_pair(1024, 1024, 192, seed=0)
m.load_images(left, right)
fl, fr = m.features()
for name, arr in list(sets.items()) + [("tower features L", None), ("tower features R", None)]:
    x = torch.from_numpy(arr).cuda() if arr is not None else (fl if name.endswith("L") else fr).reshape(-1)
    nbad = torch.zeros(1, dtype=torch.int32, device="cuda")
    first = torch.zeros(6, dtype=torch.int32, device="cuda")
    assert lib.split_probe(x.data_ptr(), x.numel(), nbad.data_ptr(), first.data_ptr(),
                           torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    f = [hex(v & 0xFFFFFFFF) for v in first.cpu().tolist()]
    print(f"{name:26s} values {x.numel():10d}  differing {int(nbad.item()):8d}  first {f if nbad.item() else '-'}", flush=True)
