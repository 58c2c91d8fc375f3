"""Compare one f16x3 tower layer (and the whole pair tower) of every tools/_var/libsde_*.so with
the in-tree library, bit for bit: max |diff|, count of differing values and where they sit
(output rows / columns, tile coordinates of 16 x 32 tiles).

    python tools/tower_ab_check.py [H] [layer]
"""
import ctypes
import glob
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import _lib, mc_cnn, ops  # noqa: E402

H = W = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
LAYER = int(sys.argv[2]) if len(sys.argv) > 2 else 3
L = 5
packed = torch.from_numpy(ops.pack_tower_weights(*mc_cnn.layer_lists(mc_cnn.synthetic_weights(L), L))).cuda()
hin, win = H + 6, W + 6
g = torch.Generator(device="cuda").manual_seed(1)
x = torch.rand((4, hin, win, 16), device="cuda", generator=g)   # c-block layout [4][h][w][16]
P, I = ctypes.c_void_p, ctypes.c_int
here = os.path.dirname(os.path.abspath(__file__))
sos = [_lib.LIB] + sorted(glob.glob(os.path.join(here, "_var", "libsde_*.so")))
# the reference: SDE_AB_REF (a library name) if given, else the in-tree library
_ref = os.environ.get("SDE_AB_REF")
if _ref:
    sos.sort(key=lambda p: os.path.basename(p) != _ref)
imgs = torch.randn((2, H + 2 * L, W + 2 * L), device="cuda", generator=g)
nws = ops.tower_batch_workspace_bytes(H, W, 2, L)
ref = None
for so in sos:
    lib = ctypes.CDLL(so)
    lib.sde_tower_layer_scaled.argtypes = [P, I, I, P, I, I, I, P, I, P, P, P, P, P, P]
    lib.sde_tower_forward_batch.argtypes = [P, I, I, I, P, I, I, P, P, ctypes.c_int64, I, P, P, P, P]
    words = torch.zeros(2, device="cuda")
    words[0] = x.abs().max()
    y = torch.full((4, hin - 2, win - 2, 16), float("nan"), device="cuda")
    s = torch.cuda.current_stream().cuda_stream
    rc = lib.sde_tower_layer_scaled(x.data_ptr(), hin, win, packed.data_ptr(), L, 64, LAYER, y.data_ptr(),
                                    8 | 2 | 4, None, None, None, words.data_ptr(), words.data_ptr() + 4, s)
    assert rc == 0, rc
    ws = torch.empty(nws, dtype=torch.uint8, device="cuda")
    feat = torch.full((2, H, W, 64), float("nan"), device="cuda")
    rc = lib.sde_tower_forward_batch(imgs.data_ptr(), 2, H, W, packed.data_ptr(), L, 64, feat.data_ptr(),
                                     ws.data_ptr(), nws, 8, None, None, None, s)
    assert rc == 0, rc
    torch.cuda.synchronize()
    name = os.path.basename(so)
    if ref is None:
        ref = (y.clone(), words.clone(), feat.clone())
        print(f"{name}: layer {LAYER} nan {int(torch.isnan(y).sum())}, bound word {words[1].item():.6g}", flush=True)
        continue
    for what, a, b in (("layer", y, ref[0]), ("pair tower", feat, ref[2])):
        d = (a - b).abs()
        bad = ~(a == b)
        n = int(bad.sum())
        msg = f"{name}: {what} differing {n}, max |diff| {float(d[~torch.isnan(d)].max()) if n else 0:.3g}"
        if n:
            idx = bad.nonzero()
            rows = idx[:, -3] if what == "layer" else idx[:, 1]
            cols = idx[:, -2] if what == "layer" else idx[:, 2]
            msg += (f"; rows {int(rows.min())}..{int(rows.max())}, cols {int(cols.min())}..{int(cols.max())}, "
                    f"tiles (y) {sorted(set((rows // 16).tolist()))[:8]} (x) {sorted(set((cols // 32).tolist()))[:8]}"
                    f", first {idx[0].tolist()}")
        print(msg, flush=True)
        if n and what == "layer":
            tx_n = (win - 2 + 31) // 32
            tiles = sorted(set(((rows // 16) * tx_n + cols // 32).tolist()))
            print(f"   bad tiles {len(tiles)}: {tiles[:40]} ... blocks(mod 512) {sorted(set(t % 512 for t in tiles))[:60]}",
                  flush=True)
            r16 = sorted(set((rows % 16).tolist()))
            c32 = sorted(set((cols % 32).tolist()))
            print(f"   rows%16 {r16} cols%32 {c32}", flush=True)
            ch = idx[:, 0] * 16 + idx[:, -1]      # c-block layout [4][h][w][16]
            print(f"   channels {sorted(set(ch.tolist()))}", flush=True)
            print(f"   tile k (t // 512): {sorted(set(t // 512 for t in tiles))}; bad tiles per k "
                  f"{[sum(1 for t in tiles if t // 512 == k) for k in range(5)]}", flush=True)
            b0 = bad[:, :16 * ((hin - 2) // 16)].reshape(4, -1, 16, win - 2, 16)
            per_tile = b0.sum(dim=(0, 2, 4))      # [tile rows][cols]
            print(f"   bad values in the first bad tile row: {per_tile[int(rows.min()) // 16].nonzero().flatten().tolist()[:40]}",
                  flush=True)
    print(f"{name}: bound word {words[1].item():.6g} vs {ref[1][1].item():.6g}", flush=True)
