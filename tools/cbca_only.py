"""CBCA kernels alone at a given size (for rocprofv3 --kernel-trace --stats)."""
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import ops  # noqa: E402


def main(H=1024, W=1024, D=192, L1=14, reps=5):
    cv = torch.randn((H, W, D), device="cuda")
    tmp = torch.empty_like(cv)
    zimg = torch.randn((H, W), device="cuda") * 0.05
    arms = ops.cbca_arms(zimg, L1, 0.02)
    for _ in range(reps):
        ops.cbca(cv, arms, arms, "left", L1, 1, tmp=tmp)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
