"""HBM traffic per launch of bench.py's dominant kernel, from rocprofv3 PMC counters.

Run on the GPU box (two separate --pmc passes, as MI355X_MICROARCH.md prescribes: FETCH_SIZE
and WRITE_SIZE do not fit one pass), then summarise:

    python tools/pmc_traffic.py run  <workload> <outdir>     # runs the two rocprofv3 passes
    python tools/pmc_traffic.py sum  <workload> <outdir> <profiles/rNN/traffic.json>

FETCH_SIZE / WRITE_SIZE are in KiB.  On gfx950 FETCH_SIZE counts half the bytes of a wide
coalesced streaming read (MI355X_MICROARCH.md, HBM section), so it is doubled; WRITE_SIZE is
exact for 16-B-per-lane streaming stores.  (Calibrated here on the CBCA horizontal pass, which
reads and writes exactly 4 B per voxel: 2 x FETCH_SIZE and WRITE_SIZE both came out at the
805 MB of the 1024x1024x192 volume.)
"""
import csv
import collections
import json
import os
import subprocess
import sys

KERNELS = {   # workload -> substring of the dominant kernel's name in the counter CSV
    "north_star": "conv64_h16_kernel<false, true, true, false, false, false, false>",
    "cones": "conv64_h16_kernel<false, true, true, false, false, false, false>",
    "cv": "cv_wta_row_kernel",
    "north_star_sgm": "sgm_scan_kernel",
    "c3": "sgm_scan_kernel",
}


def run(workload, outdir):
    for name, counters in (("fetch", ["FETCH_SIZE"]), ("write", ["WRITE_SIZE"])):
        cmd = ["rocprofv3", "--kernel-trace", "--pmc", *counters, "-d", os.path.join(outdir, name), "-o", "run",
               "--output-format", "csv", "--", sys.executable, "bench.py", "--workload", workload, "--steps", "2",
               "--warmup", "1", "--no-cpu-baseline"]
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600)


def summarise(workload, outdir, dst):
    key = KERNELS[workload]
    vals = collections.defaultdict(list)
    for name in ("fetch", "write"):
        for root, _, files in os.walk(os.path.join(outdir, name)):
            for f in files:
                if f.endswith("counter_collection.csv"):
                    for r in csv.DictReader(open(os.path.join(root, f))):
                        if key in r["Kernel_Name"]:
                            vals[(r["Counter_Name"], r.get("Dispatch_Id", ""))].append(float(r["Counter_Value"]))
    per = collections.defaultdict(list)
    for (cname, _), v in vals.items():
        per[cname].append(sum(v))          # sum over the XCD/instance rows of one dispatch
    fetch = sorted(per["FETCH_SIZE"])[len(per["FETCH_SIZE"]) // 2] * 1024 * 2
    write = sorted(per["WRITE_SIZE"])[len(per["WRITE_SIZE"]) // 2] * 1024
    out = {}
    if os.path.exists(dst):
        out = json.load(open(dst))
    out[workload] = {"kernel": key, "fetch_bytes": fetch, "write_bytes": write, "traffic_bytes": fetch + write,
                     "launches_sampled": len(per["FETCH_SIZE"]),
                     "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over "
                               "`bench.py --steps 2 --warmup 1`; median dispatch; FETCH_SIZE KiB x 2 (gfx950 "
                               "half-count of wide reads), WRITE_SIZE KiB x 1"}
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out[workload]))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        summarise(sys.argv[2], sys.argv[3], sys.argv[4])
