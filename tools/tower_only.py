"""MC-CNN tower alone at a given size (for rocprofv3 --kernel-trace --stats / --pmc)."""
import sys
import os

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import mc_cnn, ops  # noqa: E402


def main(H=1024, W=1024, reps=3, precision="bf16x6"):
    L = 5
    hw, hb = mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L)
    packed = torch.from_numpy(ops.pack_tower_weights(hw, hb)).cuda()
    img = torch.randn((H + 2 * L, W + 2 * L), device="cuda")
    out = torch.empty((H, W, 64), device="cuda")
    ws = torch.empty(ops.tower_workspace_bytes(H, W, L), dtype=torch.uint8, device="cuda")
    for _ in range(int(reps)):
        ops.tower_forward(img, packed, L, 64, out=out, workspace=ws, precision=precision)
    torch.cuda.synchronize()


if __name__ == "__main__":
    a = sys.argv[1:]
    main(*(int(x) for x in a[:3]), *a[3:4])
