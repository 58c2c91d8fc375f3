"""Why does the same SGM pair run 5.3 ms with one set of volumes and 5.8 ms with another (tools/sgm_pitch_probe.py:
W = 1024 twice in one process, 5.76 then 5.33 ms)?  Rounds of: allocate the four [1024][1024][192] volumes (cost L/R,
S L/R) a given way, time the 7-launch sde_sgm_8path_wta_pair (median of 5), print the virtual addresses (mod 1 GiB
and 2 MiB), free.  Ways: torch.empty each (the caching allocator's fresh segments, `empty_cache` between rounds),
one 4-volume block, each volume rounded up to a 1 GiB allocation."""
import ctypes
import statistics
import sys

import torch

sys.path.insert(0, ".")
from scenedepthestimation_amd import _lib, ops  # noqa: E402

H, W, D = 1024, 1024, 192
V = H * W * D * 4
GiB, MiB = 1 << 30, 1 << 20
g = torch.Generator(device="cuda").manual_seed(0)
src = [torch.rand((H, W, D), device="cuda", generator=g) for _ in range(2)]
img = [torch.randint(0, 256, (H, W), device="cuda", generator=g, dtype=torch.uint8) for _ in range(2)]
pen = [ops.sgm_penalties(i) for i in img]
disp = [torch.empty((H, W), device="cuda") for _ in range(2)]
lib = _lib.lib
s = torch.cuda.current_stream().cuda_stream
P = ctypes.c_void_p


def timed(vols):
    """vols: the four [H][W][D] float32 tensors (cost L, S L, cost R, S R)."""
    vols[0].copy_(src[0])
    vols[2].copy_(src[1])
    cl, sl, cr, sr = [v.data_ptr() for v in vols]

    def run():
        assert lib.sde_sgm_8path_wta_pair(P(cl), P(pen[0].data_ptr()), P(sl), P(disp[0].data_ptr()), P(cr),
                                          P(pen[1].data_ptr()), P(sr), P(disp[1].data_ptr()), H, W, D, 2, P(s)) == 0
    run()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return statistics.median(ts)


def show(way, vols, ms):
    ptrs = [v.data_ptr() for v in vols]
    print(f"{way:10s} {ms:7.3f} ms   VA mod 1G: " + " ".join(f"{p % GiB >> 20:5d}M" for p in ptrs) +
          "   mod 2M: " + " ".join(f"{p % (2 * MiB) >> 10:5d}K" for p in ptrs), flush=True)


def vol(t, off=0):
    return t.view(torch.uint8)[off:off + V].view(torch.float32).view(H, W, D)


for rnd in range(4):
    # separate torch allocations (what pipeline.py does)
    ts_ = [torch.empty((H, W, D), dtype=torch.float32, device="cuda") for _ in range(4)]
    show("separate", ts_, timed(ts_))
    del ts_
    torch.cuda.empty_cache()
    # one block
    blk = torch.empty(4 * V, dtype=torch.uint8, device="cuda")
    vs = [vol(blk, k * V) for k in range(4)]
    show("block", vs, timed(vs))
    del blk, vs
    torch.cuda.empty_cache()
    # 1 GiB each
    gb = [torch.empty(GiB, dtype=torch.uint8, device="cuda") for _ in range(4)]
    vs = [vol(t) for t in gb]
    show("1GiB", vs, timed(vs))
    del gb, vs
    torch.cuda.empty_cache()
    # a shifting spacer before separate allocations
    spacer = torch.empty((rnd + 1) * 37 * MiB, dtype=torch.uint8, device="cuda")
    ts_ = [torch.empty((H, W, D), dtype=torch.float32, device="cuda") for _ in range(4)]
    show("spaced", ts_, timed(ts_))
    del ts_, spacer
    torch.cuda.empty_cache()
