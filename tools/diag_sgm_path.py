"""Stage-by-stage GPU vs oracle comparison of the GPU path for one side (diagnostic)."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
import oracle  # noqa: E402
from scenedepthestimation_amd import ops  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402
from scenedepthestimation_amd.synthetic import stereo_pair  # noqa: E402

H, W, D = (int(v) for v in sys.argv[1:4])
side = int(sys.argv[4]) if len(sys.argv) > 4 else 1
oracle.set_threads(16)
left, right, _ = stereo_pair(H, W, D, seed=4)
m = StereoMatcher(H, W, D, sgm=True, cbca_iters=2)
m.load_images(left, right)
m.features()
b = m.sgm_bufs
ops.cost_volume(m.feat[0], m.feat[1], D, layout="HWD", right=True, invalid=1.0, out_left=b["cv"][0], out_right=b["cv"][1])
h = lambda t: (torch.cuda.synchronize(), t.cpu().numpy())[1]
fl, fr = h(m.feat[0]), h(m.feat[1])
t = time.time()
cl, cr = oracle.cost_volume_hwd(fl, fr, D, invalid=1.0, right=True)
print("oracle cv", time.time() - t, flush=True)
g = [h(b["cv"][0]), h(b["cv"][1])]
o = [cl, cr]
for k in range(2):
    print("cv side", k, "mismatch voxels", int((g[k].view(np.int32) != o[k].view(np.int32)).sum()), flush=True)
m.cbca(b["cv"][0], b["cv"][1], m.img_u8[0], m.img_u8[1])
P = m.nlayers
zl = h(m.img_pad[0])[P:P + H, P:P + W]
zr = h(m.img_pad[1])[P:P + H, P:P + W]
al, ar = oracle.cbca_arms(zl), oracle.cbca_arms(zr)
print("arms", np.array_equal(h(b["arms"][0]).view(np.uint32), al), np.array_equal(h(b["arms"][1]).view(np.uint32), ar))
o = [oracle.cbca(cl, al, ar, "left", 2), oracle.cbca(cr, ar, al, "right", 2)]
g = [h(b["cv"][0]), h(b["cv"][1])]
for k in range(2):
    bad = g[k].view(np.int32) != o[k].view(np.int32)
    print("cbca side", k, "mismatch voxels", int(bad.sum()), flush=True)
    if bad.any():
        idx = np.argwhere(bad)
        print("  first", idx[:5].tolist(), "rows", np.unique(idx[:, 0])[:10].tolist(), "cols", np.unique(idx[:, 1])[:10].tolist(),
              "d", np.unique(idx[:, 2])[:10].tolist())
        y, x, d = idx[0]
        print("  gpu", g[k][y, x, d], "oracle", o[k][y, x, d])
pens = [ops.sgm_penalties(m.img_u8[0]), ops.sgm_penalties(m.img_u8[1])]
for k in range(2):
    S = torch.empty_like(b["cv"][k])
    ops.sgm_8path_pair(b["cv"][k], pens[k], S, zero_du_penalties=True)
    So = oracle.sgm_8path(o[k], oracle.sgm_penalties([left, right][k]))
    Sg = h(S)
    bad = Sg.view(np.int32) != So.view(np.int32)
    print("sgm side", k, "mismatch", int(bad.sum()), flush=True)
    if bad.any():
        idx = np.argwhere(bad)
        print("  first", idx[:5].tolist(), "rows", np.unique(idx[:, 0])[:10].tolist())
# the product path: fused WTA + post-processing
dl, dr = m.sgm_path(post=False)
wl = oracle.wta_sgm(oracle.sgm_8path(o[0], oracle.sgm_penalties(left)))
wr = oracle.wta_sgm(oracle.sgm_8path(o[1], oracle.sgm_penalties(right)))
for k, (gd, od) in enumerate(((h(dl), wl), (h(dr), wr))):
    bad = gd != od
    print("fused wta side", k, "mismatch px", int(bad.sum()), flush=True)
    if bad.any():
        idx = np.argwhere(bad)
        print("  first", idx[:8].tolist(), "rows", np.unique(idx[:, 0])[:10].tolist(), "cols", np.unique(idx[:, 1])[:10].tolist())
        y, x = idx[0]
        print("  gpu", gd[y, x], "oracle", od[y, x])
dl, dr = m.sgm_path(post=True)
a, _ = oracle.lr_check(wl, wr)
for k, (gd, od) in enumerate(((h(dl), oracle.median5(oracle.lrc_fill(wl, a), wl)), (h(dr), oracle.median5(wr, wr)))):
    bad = gd != od
    print("post side", k, "mismatch px", int(bad.sum()), flush=True)
    if bad.any():
        idx = np.argwhere(bad)
        print("  first", idx[:8].tolist())
        y, x = idx[0]
        print("  gpu", gd[y, x], "oracle", od[y, x])
