"""Run the f16x3 tower pair (1024^2, 5 layers) back to back for argv[1] seconds (tools/power_probe.sh)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import mc_cnn, ops  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
H = W = 1024
L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
imgs = torch.randn((2, H + 2 * L, W + 2 * L), device="cuda")
feat = torch.empty((2, H, W, 64), device="cuda")
ws = torch.empty(ops.tower_batch_workspace_bytes(H, W, 2, L), dtype=torch.uint8, device="cuda")
t0 = time.time()
n = 0
while time.time() - t0 < secs:
    for _ in range(50):
        ops.tower_forward_batch(imgs, packed, L, out=feat, workspace=ws)
    torch.cuda.synchronize()
    n += 50
    print(f"{time.time() - t0:6.1f} s  {n} pairs  {(time.time() - t0) / n * 1e3:.3f} ms/pair", flush=True)
