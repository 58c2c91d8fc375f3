"""Is the SGM pair's process-to-process spread (LR/RL 0.80 vs 0.95 ms per launch) a state of
the box rather than of the code?  One process, one set of buffers, the same 7-launch sde_sgm_8path_wta_pair at
1024^2 x 192 timed (HIP events, median of 5 pairs) at several points:
  cold      first thing after allocation (the box idle before this process)
  hbm_hot   after ~10 s of back-to-back SGM pairs (HBM streaming at ~5.5 TB/s)
  rest      after 20 s idle
  mfma_hot  after ~10 s of back-to-back tower layers (MFMA-bound, little HBM traffic)
  rest2     after 20 s idle again
The per-launch split comes from running this script under rocprofv3 --kernel-trace."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import mc_cnn, ops  # noqa: E402

H, W, D = 1024, 1024, 192
g = torch.Generator(device="cuda").manual_seed(0)
cv = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
S = [torch.empty((H, W, D), device="cuda") for _ in range(2)]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
x = torch.rand((2, H + 6, W + 6, 64), device="cuda")
y = torch.empty((2, H + 4, W + 4, 64), device="cuda")
words = torch.ones(4, device="cuda")


def pair():
    ops.sgm_8path_wta_pair(cv[0], pen[0], S[0], disp[0], cv[1], pen[1], S[1], disp[1], zero_du_penalties=True)


def tower_layer():
    ops.tower_layer_batch(x, packed, L, 3, y, in_cblock=True, out_cblock=True, in_absmax=words[0:1],
                          out_absmax=words[1:2])


def timed(fn, n=5):
    ts = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts), ts


def burn(fn, seconds):
    t0 = time.time()
    n = 0
    while time.time() - t0 < seconds:
        for _ in range(10):
            fn()
        torch.cuda.synchronize()
        n += 10
    return n


def point(name):
    m, ts = timed(pair)
    print(f"{name:9s} SGM pair {m:7.3f} ms   ({' '.join(f'{t:.3f}' for t in ts)})", flush=True)


point("cold")
print(f"  burn: {burn(pair, 10)} SGM pairs", flush=True)
point("hbm_hot")
time.sleep(20)
point("rest")
print(f"  burn: {burn(tower_layer, 10)} tower layers", flush=True)
point("mfma_hot")
time.sleep(20)
point("rest2")
