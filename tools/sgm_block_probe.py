"""The four SGM volumes (cost L, S L, cost R, S R; 768 MiB each at 1024^2 x 192) carved out of ONE allocation
at offsets k * (V + delta) for a range of deltas: the 7-launch sde_sgm_8path_wta_pair timed per layout (median of
5), rounds over fresh allocations.  Separate allocations run 5.3 or 5.8 ms by placement (tools/sgm_alloc_probe.py);
a block with delta = 0 always ran ~5.8: is the spacing what decides?"""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import _lib, ops  # noqa: E402
import ctypes

H, W, D = 1024, 1024, 192
V = H * W * D * 4
MiB = 1 << 20
deltas = [int(x) * MiB for x in sys.argv[1].split(",")] if len(sys.argv) > 1 else \
    [x * MiB for x in (0, 1, 2, 16, 64, 96, 128, 192, 256, 320, 384, 512)]
g = torch.Generator(device="cuda").manual_seed(0)
src = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
lib = _lib.lib
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p
res = {}
for rnd in range(2):
    for dl in deltas:
        blk = torch.empty(4 * V + 3 * dl, dtype=torch.uint8, device="cuda")
        vs = [blk[k * (V + dl):k * (V + dl) + V].view(torch.float32).view(H, W, D) for k in range(4)]
        vs[0].copy_(src[0])
        vs[2].copy_(src[1])
        cl, sl, cr, sr = [v.data_ptr() for v in vs]

        def run():
            assert lib.sde_sgm_8path_wta_pair(P(cl), P(pen[0].data_ptr()), P(sl), P(disp[0].data_ptr()), P(cr),
                                              P(pen[1].data_ptr()), P(sr), P(disp[1].data_ptr()), H, W, D, 2,
                                              P(s)) == 0
        run()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        res.setdefault(dl, []).append(statistics.median(ts))
        print(f"round {rnd} delta {dl // MiB:4d} MiB: {statistics.median(ts):7.3f} ms", flush=True)
        del blk, vs
        torch.cuda.empty_cache()
for dl, v in res.items():
    print(f"delta {dl // MiB:4d} MiB: " + " ".join(f"{t:.3f}" for t in v), flush=True)
