"""CBCA alone at a given size (for rocprofv3 --kernel-trace --stats): sde_cbca_lr (the GPU path's
pair: one volume aggregated, one shear) with ITERS iterations, timed with events, median of 5 rounds.

    python tools/cbca_only.py [H W D L1 ITERS REPS]
"""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import ops  # noqa: E402


def timed(fn, reps):
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main(H=1024, W=1024, D=192, L1=14, iters=2, reps=5):
    cl, cr = torch.randn((H, W, D), device="cuda"), torch.randn((H, W, D), device="cuda")
    tmp = torch.empty_like(cl)
    ws = torch.empty((ops.cbca_workspace_bytes(H, W),), dtype=torch.uint8, device="cuda")
    g = torch.Generator(device="cuda").manual_seed(0)
    blocks = torch.randint(0, 4, (H // 8 + 1, W // 8 + 1), device="cuda", generator=g).float() * 0.05
    zimg = blocks.repeat_interleave(8, 0).repeat_interleave(8, 1)[:H, :W].contiguous()
    al = ops.cbca_arms(zimg + torch.randn((H, W), device="cuda", generator=g) * 0.004, L1, 0.02)
    ar = ops.cbca_arms(zimg + torch.randn((H, W), device="cuda", generator=g) * 0.004, L1, 0.02)
    ts = [timed(lambda: ops.cbca_lr(cl, cr, al, ar, L1, iters, tmp=tmp, workspace=ws), reps) for _ in range(5)]
    ms = sorted(ts)[2]
    valid = float(H) * sum(max(W - d, 0) for d in range(D))
    gb = (16.0 * iters + 8.0) * valid / 1e6          # GB * 1e3: GB/s from ms
    print("cbca_lr:", " ".join(f"{t:.3f}" for t in ts))
    print(f"cbca_lr {iters} iterations + shear: {ms:.3f} ms = {gb / ms:.0f} GB/s algorithmic "
          f"({(16.0 * iters + 8.0) * valid / 1e9:.2f} GB)", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
