"""Run the tower's layer 3 (both images, 1024^2) N times: Winograd (arg 'wino') or direct (arg 'direct')."""
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import ops  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher, tower_steps  # noqa: E402
from scenedepthestimation_amd.synthetic import stereo_pair  # noqa: E402

direct = len(sys.argv) > 1 and sys.argv[1] == "direct"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H = W = 1024
left, right, _ = stereo_pair(H, W, 192, seed=0)
m = StereoMatcher(H, W, 192)
m.load_images(left, right)
m.features()
L = 5
hin, win = H + 2 * L - 4, W + 2 * L - 4
act = hin * win * 64
wsf = m.ws.view(torch.float32)
src = wsf[:2 * act].view(2, hin, win, 64)
dst = wsf[2 * act:2 * act + 2 * (hin - 2) * (win - 2) * 64].view(2, hin - 2, win - 2, 64)
words = torch.ones((2, 64), dtype=torch.float32, device="cuda")
for _ in range(n):
    ops.tower_layer_batch(src, m.packed, L, 3, dst, precision="f16x3" if direct else "f16x3w", in_cblock=True,
                          out_cblock=True, in_absmax=words[:, 0:1], out_absmax=words[:, 1:2])
torch.cuda.synchronize()
print("ok")
