"""CBCA passes' rate by volume shape at a fixed voxel count (~201 M): does a wave's 256-B run per step cost more
when a pixel's disparities span several waves (D = 192: 3 chunks, 768-B pixel runs) than when one wave covers the
pixel (D = 64)?  Times sde_cbca_lr (2 iterations + shear) and prints GB/s on the v2 algorithmic bytes."""
import statistics
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import ops  # noqa: E402

for (H, W, D) in [(1024, 1024, 192), (1024, 3072, 64), (3072, 1024, 64), (1024, 1536, 128), (512, 1024, 384)]:
    g = torch.Generator(device="cuda").manual_seed(0)
    cl = torch.rand((H, W, D), device="cuda", generator=g)
    cr = torch.empty_like(cl)
    tmp = torch.empty_like(cl)
    img = [torch.rand((H, W), device="cuda", generator=g) for _ in range(2)]
    arms = [ops.cbca_arms(i) for i in img]
    ws = torch.empty(ops.cbca_workspace_bytes(H, W), dtype=torch.uint8, device="cuda")

    def run():
        ops.cbca_lr(cl, cr, arms[0], arms[1], 14, 2, tmp=tmp, workspace=ws)
    run()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ms = statistics.median(ts)
    valid = float(H) * sum(max(W - d, 0) for d in range(D))
    print(f"{H}x{W}x{D}: cbca_lr {ms:.3f} ms  {(40.0 * valid) / (ms * 1e-3) / 1e9:.0f} GB/s  ({H * W * D / 1e6:.0f} Mvox)",
          flush=True)
    del cl, cr, tmp, ws
    torch.cuda.empty_cache()
