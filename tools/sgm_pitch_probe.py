"""Does the SGM pair's speed depend on the volumes' row stride (DRAM channel / bank mapping of 2048 lock-step
row streams)?  The 7-launch sde_sgm_8path_wta_pair at H = 1024, D = 192 for widths W in a list (row stride
W * 768 B: W = 1024 is 3 * 2^18 B), timed with HIP events (median of 5 pairs) and normalised per voxel to
W = 1024.  Run under rocprofv3 --kernel-trace for the per-launch (per-direction) split."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import ops  # noqa: E402

H, D = 1024, 192
widths = [int(w) for w in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1024, 1025, 1032, 1040, 1088, 1008]
g = torch.Generator(device="cuda").manual_seed(0)
for W in widths:
    cv = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
    img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
    pen = [ops.sgm_penalties(i) for i in img]
    S = [torch.empty((H, W, D), device="cuda") for _ in range(2)]
    disp = [torch.empty((H, W), device="cuda") for _ in range(2)]

    def pair():
        ops.sgm_8path_wta_pair(cv[0], pen[0], S[0], disp[0], cv[1], pen[1], S[1], disp[1], zero_du_penalties=True)
    pair()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        pair()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    m = statistics.median(ts)
    print(f"W={W:5d} stride {W * D * 4:9d} B  pair {m:7.3f} ms  per 1024^2 {m * 1024 / W:7.3f} ms", flush=True)
    del cv, S, pen, disp
    torch.cuda.empty_cache()
