"""Does a tower layer run faster when its input activations are served from the 256 MiB Infinity Cache
instead of HBM?  (The tower is power-capped -- DESIGN.md sec. 3.2 -- and MI355X holds a higher clock for the
same MFMAs when their streamed data comes from on-die caches; cdna_hip_programming.md sec. 5.4 rule 28.)

One middle layer (layer 3, f16x3, c-block layouts) on one image of H rows x 1026 columns (32 tile columns,
so H = 2 + 128 k gives exactly k rounds of 256 tiles: no tail):
  warm -- launches back to back: the input (H x 1026 x 256 B) and output stay in the Infinity Cache when
          they fit (H = 386: 101 + 100 MB);
  cold -- the same launches with 640 MB of other traffic (a copy) between them, outside the timed events.
Per-round times compare sizes that fit the cache with sizes that do not.  usage: python tools/mall_probe.py [H ...]"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import mc_cnn, ops  # noqa: E402

L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
junk_a = torch.empty(160 << 20, device="cuda")          # 640 MB
junk_b = torch.empty_like(junk_a)
Ws = 1026
for H in [int(a) for a in sys.argv[1:]] or [130, 258, 386, 514, 1026]:
    x = torch.rand((H, Ws, 64), device="cuda")
    y = torch.empty((H - 2, Ws - 2, 64), device="cuda")
    words = torch.ones(2, device="cuda")

    def layer():
        ops.tower_layer(x, packed, L, 3, y, precision="f16x3", in_cblock=True, out_cblock=True,
                        in_absmax=words[0:1], out_absmax=words[1:2])
    res = {}
    for rnd in range(3):
        for arm in ("warm", "cold"):
            ts = []
            for _ in range(8):
                if arm == "cold":
                    junk_b.copy_(junk_a)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                layer()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            res.setdefault(arm, []).append(statistics.median(ts[2:]))
    w, c = statistics.median(res["warm"]), statistics.median(res["cold"])
    mb = H * Ws * 256 / 1e6
    rounds = (H - 2) // 128
    print(f"H={H:5d} (input {mb:6.1f} MB, {rounds} rounds): warm {w:7.1f} us  cold {c:7.1f} us  warm/cold {w / c:.3f}"
          f"   per round warm {w / rounds:6.1f} cold {c / rounds:6.1f} us", flush=True)
