"""Run only the fused CV+WTA kernels (both modes) a few times at 1024x1024x192 (profiling driver)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import ops  # noqa: E402
from scenedepthestimation_amd.synthetic import features  # noqa: E402

H, W, D = (int(a) for a in (sys.argv[1:4] if len(sys.argv) > 3 else (1024, 1024, 192)))
modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["certified", "exact"]
fl = torch.from_numpy(features(H, W, seed=0)).cuda()
fr = torch.from_numpy(features(H, W, seed=1)).cuda()
ws = torch.empty(ops.cv_wta_workspace_bytes(H, W), dtype=torch.uint8, device="cuda")
disp = torch.empty((H, W), device="cuda")
for mode in modes:
    for _ in range(3):
        ops.cv_wta(fl, fr, 0, D, disp=disp, want=(), mode=mode, workspace=ws)
torch.cuda.synchronize()
print("fixups", ops.cv_wta_fixups(ws))
