"""Probe of the SGM pair's process-to-process spread ("LR/RL 0.80 vs 0.95 ms"): the
7-launch sde_sgm_8path_wta_pair at 1024^2 x 192 timed with HIP events in THIS process for the in-tree
library and the tools/_var/libsde_sgmgap*.so probe builds (SRC=tools/variants/sgm_probe.hip bash
tools/build_file_variant.sh sgm.hip sgmgapN -DSGM_GAP=N; SGM_GAP: 1 = host sync between passes,
2 = an event record with a system-scope release between passes, 3 = a plain event record), round-robin,
median of 7.  The per-launch split comes from a rocprofv3 --kernel-trace run of this same script."""
import ctypes
import glob
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib, ops  # noqa: E402

H, W, D = 1024, 1024, 192
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
g = torch.Generator(device="cuda").manual_seed(0)
cv = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
S = [torch.empty((H, W, D), device="cuda") for _ in range(2)]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
P, I = ctypes.c_void_p, ctypes.c_int
here = os.path.dirname(os.path.abspath(__file__))
sos = [_lib.LIB] + sorted(glob.glob(os.path.join(here, "_var", "libsde_sgmgap*.so")))
libs = []
for so in sos:
    lib = ctypes.CDLL(so)
    lib.sde_sgm_8path_wta_pair.argtypes = [P] * 8 + [I, I, I, I, P]
    libs.append((os.path.basename(so), lib))
s = torch.cuda.current_stream().cuda_stream


def run(lib):
    assert lib.sde_sgm_8path_wta_pair(cv[0].data_ptr(), pen[0].data_ptr(), S[0].data_ptr(), disp[0].data_ptr(),
                                      cv[1].data_ptr(), pen[1].data_ptr(), S[1].data_ptr(), disp[1].data_ptr(),
                                      H, W, D, 2, s) == 0


def timed(lib, n):
    run(lib)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        run(lib)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


ref = None
ok_libs = []
for name, lib in libs:
    try:
        run(lib)
    except AssertionError:
        print(f"{name:24s} FAILED (status != 0): skipped", flush=True)
        continue
    torch.cuda.synchronize()
    o = [d.clone() for d in disp]
    ref = ref or o
    ok_libs.append((name, lib))
    print(f"{name:24s} disparities identical: {all(torch.equal(a, b) for a, b in zip(o, ref))}", flush=True)
libs = ok_libs
res = {}
for rnd in range(7):
    for name, lib in libs:
        res.setdefault(name, []).append(timed(lib, reps))
for name, v in res.items():
    print(f"{name:24s} pair {statistics.median(v):7.3f} ms   ({' '.join(f'{t:.3f}' for t in v)})", flush=True)
