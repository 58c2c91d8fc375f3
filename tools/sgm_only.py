"""Run sde_sgm_8path_wta_pair (both sides, 1024^2 x 192, synthetic costs) N times (PMC / trace driver)."""
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import ops  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 3
H, W, D = 1024, 1024, 192
g = torch.Generator(device="cuda").manual_seed(0)
cv = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
S = [torch.empty((H, W, D), device="cuda") for _ in range(2)]
for _ in range(n):
    ops.sgm_8path_wta_pair(cv[0], pen[0], S[0], None, cv[1], pen[1], S[1], None, zero_du_penalties=True)
torch.cuda.synchronize()
print("ok")
