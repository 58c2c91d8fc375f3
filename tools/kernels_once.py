"""Each north-star kernel twice at 1024x1024, D = 192 (PMC traffic driver, tools/pmc_traffic_kernels.py):
the tower (f16x3, both images per launch), the certified CV+WTA, the left volume (the aggregation
path's cost-volume sweep), sde_cbca_lr at 2 iterations and the 7-launch SGM pair + WTA."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402
from scenedepthestimation_amd import ops  # noqa: E402
from scenedepthestimation_amd.synthetic import stereo_pair  # noqa: E402

H, W, D = 1024, 1024, 192
left, right, _ = stereo_pair(H, W, D, seed=0)
m = StereoMatcher(H, W, D, sgm=True, cbca_iters=2)
m.load_images(left, right)
b = m.sgm_bufs
for _ in range(2):
    m.features()
    m.cost_wta()
    ops.cost_volume(m.feat[0], m.feat[1], D, layout="HWD", invalid=1.0, out_left=b["cv"][0])
    m.cbca(b["cv"][0], b["cv"][1], m.img_u8[0], m.img_u8[1])
    ops.sgm_penalties(m.img_u8[0], out=b["pen"][0])
    ops.sgm_penalties(m.img_u8[1], out=b["pen"][1])
    ops.sgm_8path_wta_pair(b["cv"][0], b["pen"][0], b["S"][0], b["disp"][0], b["cv"][1], b["pen"][1], b["S"][1],
                           b["disp"][1], zero_du_penalties=True)
torch.cuda.synchronize()
print("ok")
