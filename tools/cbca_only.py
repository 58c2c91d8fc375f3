"""CBCA kernels alone at a given size (for rocprofv3 --kernel-trace --stats): one iteration of
both sides as two single-volume calls, then as one sde_cbca_pair call, each timed with events."""
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


def main(H=1024, W=1024, D=192, L1=14, reps=5):
    cl, cr = torch.randn((H, W, D), device="cuda"), torch.randn((H, W, D), device="cuda")
    tl, tr = torch.empty_like(cl), torch.empty_like(cl)
    g = torch.Generator(device="cuda").manual_seed(0)
    blocks = torch.randint(0, 4, (H // 8 + 1, W // 8 + 1), device="cuda", generator=g).float() * 0.05
    zimg = blocks.repeat_interleave(8, 0).repeat_interleave(8, 1)[:H, :W].contiguous()
    al = ops.cbca_arms(zimg + torch.randn((H, W), device="cuda", generator=g) * 0.004, L1, 0.02)
    ar = ops.cbca_arms(zimg + torch.randn((H, W), device="cuda", generator=g) * 0.004, L1, 0.02)

    def single():
        ops.cbca(cl, al, ar, "left", L1, 1, tmp=tl)
        ops.cbca(cr, ar, al, "right", L1, 1, tmp=tr)
    ss, ps = [], []
    for _ in range(5):      # interleaved: the clock drifts over a run
        ss.append(timed(single, reps))
        ps.append(timed(lambda: ops.cbca_pair(cl, cr, al, ar, L1, 1, tmp_l=tl, tmp_r=tr), reps))
    ms_s, ms_p = sorted(ss)[2], sorted(ps)[2]
    print("single:", " ".join(f"{t:.3f}" for t in ss), " pair:", " ".join(f"{t:.3f}" for t in ps))
    gb = 2 * 16 * H * W * D / 1e6     # GB * 1e3: GB/s from ms
    print(f"one iteration, both sides: two single calls {ms_s:.3f} ms ({gb / ms_s:.0f} GB/s), "
          f"pair {ms_p:.3f} ms ({gb / ms_p:.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
