"""Does the order of a pair's kernels matter under the power cap?  The tower layers run at the board's power
cap; the certified CV+WTA does not (latency-bound).  One stream, no concurrency: the CV+WTA of pair k - 1 is
issued between two tower layers of pair k (two StereoMatchers, the same images) instead of after the tower of
its own pair.  Same kernels, same work per pair; only their order changes.
usage: python tools/interleave_probe.py"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import stereo_pair  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402

H, W, D = 1024, 1024, 192
left, right, _ = stereo_pair(H, W, D, seed=0)
ms = [StereoMatcher(H, W, D) for _ in range(2)]
for m in ms:
    m.load_images(left, right)
k = [0]


def seq():
    m = ms[k[0] % 2]
    m.features()
    m.cost_wta()
    k[0] += 1


def inter(after):
    def step():
        m, mp = ms[k[0] % 2], ms[(k[0] + 1) % 2]

        def hook(layer, launch):
            launch()
            if layer == after:
                mp.cost_wta()        # the previous pair's CV+WTA between this pair's tower layers
        m.features(on_launch=hook)
        k[0] += 1
    return step


def timed(fn, n=40):
    for _ in range(4):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


res = {}
arms = [("seq", seq), ("cv after layer 2", inter(2)), ("cv after layer 3", inter(3)), ("cv after layer 4", inter(4)),
        ("cv after layer 5", inter(5))]
for rnd in range(3):
    for name, fn in arms:
        res.setdefault(name, []).append(timed(fn))
for name, v in res.items():
    print(f"{name:18s} {statistics.median(v):7.3f} ms/pair   ({' '.join(f'{t:.3f}' for t in v)})", flush=True)
