"""Is the north-star pair throughput power-bound enough that the certified CV+WTA of pair k can run beside the
tower of pair k+1 for free?  (the tower runs at the board's power cap.)

Times, at 1024^2 x 192 with two StereoMatchers (two feature sets, the same images):
  seq        -- the bench's step: features() then cost_wta() on one stream, pair after pair;
  tower@G    -- the tower alone on a stream masked to G CUs with its grid capped at G;
  overlap@G  -- tower of pair k on a G-CU stream, CV+WTA of pair k on a stream of the other 256 - G CUs
                (events: the CV waits for its tower, a tower waits for the CV that last read its features).
CU masks: hipExtStreamCreateWithCUMask from the HIP runtime the process already loaded.
usage: python tools/overlap_probe.py [G ...]"""
import ctypes
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scenedepthestimation_amd import ops  # noqa: E402
from scenedepthestimation_amd.pipeline import StereoMatcher  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import stereo_pair  # noqa: E402


def hip_runtime():
    with open("/proc/self/maps") as fh:
        for line in fh:
            if "libamdhip64.so" in line:
                return ctypes.CDLL(line.split()[-1])
    raise RuntimeError("libamdhip64 not loaded")


H, W, D = 1024, 1024, 192
torch.zeros(1, device="cuda")
hip = hip_runtime()
ncu = torch.cuda.get_device_properties(0).multi_processor_count
left, right, _ = stereo_pair(H, W, D, seed=0)
ms = [StereoMatcher(H, W, D) for _ in range(2)]
for m in ms:
    m.load_images(left, right)


def masked_stream(bits):
    words = [0] * ((ncu + 31) // 32)
    for b in bits:
        words[b >> 5] |= 1 << (b & 31)
    arr = (ctypes.c_uint32 * len(words))(*words)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(len(words)), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value)


def timed(fn, n, streams):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for s in streams:   # the timed region starts after every stream's earlier work
        s.wait_event(e0)
    for _ in range(n):
        fn()
    for s in streams:
        ev = torch.cuda.Event()
        ev.record(s)
        torch.cuda.current_stream().wait_event(ev)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def seq():
    ms[0].match()


res = {"seq": [timed(seq, 40, [])]}
gs = [int(a) for a in sys.argv[1:]] or [224, 232, 240]
for G in gs:
    for pat in ("spread", "tail"):
        rest = [b for b in range(ncu) if (b % (ncu // (ncu - G)) == ncu // (ncu - G) - 1)] if pat == "spread" else \
            list(range(G, ncu))
        rest = rest[:ncu - G]
        tow_bits = [b for b in range(ncu) if b not in set(rest)]
        sa, sb = masked_stream(tow_bits), masked_stream(rest)
        ops.set_persistent_grid(G)

        def tower_only():
            with torch.cuda.stream(sa):
                ms[0].features()
        res.setdefault(f"tower@{G} {pat}", []).append(timed(tower_only, 40, [sa]))
        k = [0]
        ev_t = [torch.cuda.Event(), torch.cuda.Event()]
        ev_c = [torch.cuda.Event(), torch.cuda.Event()]
        for e in ev_c:
            e.record(sb)

        def overlap():
            i = k[0] % 2
            m = ms[i]
            with torch.cuda.stream(sa):
                sa.wait_event(ev_c[i])        # the CV that last read this matcher's features
                m.features()
                ev_t[i].record(sa)
            with torch.cuda.stream(sb):
                sb.wait_event(ev_t[i])
                m.cost_wta()
                ev_c[i].record(sb)
            k[0] += 1
        res.setdefault(f"overlap@{G} {pat}", []).append(timed(overlap, 40, [sa, sb]))
        ops.set_persistent_grid(0)
        # the overlapped maps equal the sequential one
        torch.cuda.synchronize()
        ref = ms[0].disp.clone()
        ms[1].match()
        torch.cuda.synchronize()
        print(f"G={G} {pat}: maps identical {torch.equal(ref, ms[1].disp)}", flush=True)
res["seq"].append(timed(seq, 40, []))
for k2, v in res.items():
    print(f"{k2:22s} {statistics.median(v):7.3f} ms/pair   ({' '.join(f'{t:.3f}' for t in v)})", flush=True)
