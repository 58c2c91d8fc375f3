"""Per-kernel PMC summary from several rocprofv3 --pmc passes (one pass per counter group).

    python tools/pmc_kernel.py run <outdir> -- <command ...>    # GPU box: runs the passes
    python tools/pmc_kernel.py sum <outdir> [kernel-substring]  # prints mean per dispatch

Counter groups respect the per-pass limits of MI355X_MICROARCH.md (<= 8 SQ, <= 2 GRBM).
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles; SQ_VALU_MFMA_BUSY_CYCLES
counts cycles; GRBM_GUI_ACTIVE sums the 8 XCDs.
"""
import collections
import csv
import os
import subprocess
import sys

GROUPS = [
    ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
     "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"],
    ["SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_SALU",
     "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "SQ_WAIT_INST_LDS"],
    ["GRBM_GUI_ACTIVE", "GRBM_COUNT", "SQ_ACTIVE_INST_VMEM", "SQ_INST_LEVEL_VMEM", "SQ_LDS_IDX_ACTIVE",
     "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_INSTS_VMEM_WR"],
]


def run(outdir, cmd):
    for i, g in enumerate(GROUPS):
        c = ["timeout", "-s", "KILL", "120", "rocprofv3", "--kernel-trace", "--pmc", *g, "-d",
             os.path.join(outdir, f"g{i}"), "-o", "run", "--output-format", "csv", "--", *cmd]
        r = subprocess.run(c, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        if r.returncode != 0:
            print(r.stderr[-2000:])
            sys.exit(r.returncode)


def summarise(outdir, key=None):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for root, _, files in os.walk(outdir):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    kn = r["Kernel_Name"]
                    if key and key not in kn:
                        continue
                    d = (root, r.get("Dispatch_Id", ""))
                    vals[(kn, r["Counter_Name"])][d] += float(r["Counter_Value"])
                    names[kn] = 1
    for kn in names:
        print(kn[:100])
        for (k2, cn), per in sorted(vals.items()):
            if k2 == kn:
                v = sorted(per.values())
                print(f"   {cn:28s} {v[len(v) // 2]:16.4g}   (median of {len(v)} dispatches)")


if __name__ == "__main__":
    if sys.argv[1] == "run":
        i = sys.argv.index("--")
        run(sys.argv[2], sys.argv[i + 1:])
    else:
        summarise(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
