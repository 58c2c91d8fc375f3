"""HBM traffic per launch of each north-star kernel from rocprofv3 PMC (FETCH_SIZE and WRITE_SIZE in
separate passes, as MI355X_MICROARCH.md prescribes) over tools/kernels_once.py.

    python tools/pmc_traffic_kernels.py run <outdir>                  # GPU box
    python tools/pmc_traffic_kernels.py sum <outdir> <profiles/rNN/traffic.json>

FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE counts half the bytes of wide coalesced streaming
reads on gfx950 (MI355X_MICROARCH.md, HBM section), so it is doubled.  Per kernel: the median
over its dispatches of the per-dispatch sum over instances; the SGM entry is the sum of its
seven launches' medians (one pair call).  Keys are what bench.py's measured_traffic() reads.
"""
import collections
import csv
import json
import os
import subprocess
import sys

KERNELS = {   # key -> (substring of the kernel name, sum over distinct names) or [(substring, dispatches per unit)]
    "tower_conv64_layer": ("conv64_h16_kernel<false, true, true, false, false, false, false>", False),
    "cv_wta_row": ("cv_wta_row2_kernel<false>", False),
    "cvlr": ("cvlr3_kernel", False),
    # one sde_cbca_lr call at 2 iterations: 2 transposes, 2 x (horizontal + vertical pass), 1 shear
    "cbca_lr": [("cbca_transpose_kernel", 2), ("cbca_h_kernel", 2), ("cbca_v_kernel", 2), ("cbca_rotate_kernel", 1)],
    "sgm_pair": ("sgm_scan_kernel", True),
}
WORKLOAD_KEYS = {"north_star": "tower_conv64_layer", "cones": None, "cv": "cv_wta_row",
                 "north_star_sgm": "sgm_pair", "c3": None}


def run(outdir):
    for name, counters in (("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE"])):
        cmd = ["timeout", "-s", "KILL", "120", "rocprofv3", "--kernel-trace", "--pmc", *counters, "-d",
               os.path.join(outdir, name), "-o", "run", "--output-format", "csv", "--", sys.executable,
               "tools/kernels_once.py"]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)


def summarise(outdir, dst):
    per = collections.defaultdict(lambda: collections.defaultdict(float))   # (counter, kernel) -> dispatch -> sum
    for name in ("fetch", "write"):
        for root, _, files in os.walk(os.path.join(outdir, name)):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    for r in csv.DictReader(open(os.path.join(root, f))):
                        per[(r["Counter_Name"], r["Kernel_Name"])][r.get("Dispatch_Id", "")] += \
                            float(r["Counter_Value"])
    med = {}
    for (cn, kn), d in per.items():
        v = sorted(d.values())
        med[(cn, kn)] = (v[len(v) // 2], len(v))
    out = {"method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/kernels_once.py "
                     "(1024x1024, D=192); median dispatch per kernel; FETCH_SIZE KiB x 2 (gfx950 half-count of "
                     "wide reads), WRITE_SIZE KiB x 1"}
    for key, spec in KERNELS.items():
        if isinstance(spec, list):
            parts = [(kn, n) for sub, n in spec for kn in sorted({kn for (_, kn) in med if sub in kn})[:1]]
            sub = " + ".join(f"{n} x {s}" for s, n in spec)
        else:
            sub, many = spec
            names = sorted({kn for (_, kn) in med if sub in kn})
            parts = [(kn, 1) for kn in (names if many else names[:1])]
        if not parts:
            continue
        fetch = sum(med.get(("FETCH_SIZE", kn), (0, 0))[0] * n for kn, n in parts) * 1024 * 2
        write = sum(med.get(("WRITE_SIZE", kn), (0, 0))[0] * n for kn, n in parts) * 1024
        out[key] = {"kernel": sub, "launches": sum(n for _, n in parts), "fetch_bytes": fetch, "write_bytes": write,
                    "traffic_bytes": fetch + write}
    for w, key in WORKLOAD_KEYS.items():
        if key and key in out:
            out[w] = dict(out[key], alias_of=key)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        summarise(sys.argv[2], sys.argv[3])
