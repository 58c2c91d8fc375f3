# HBM traffic of the L/R volume kernel (cvlr_dma_kernel) at 1024^2 x 192: FETCH_SIZE and WRITE_SIZE in
# separate rocprofv3 --pmc passes (MI355X_MICROARCH.md); summarised by tools/pmc_traffic.py's rules.
# usage: gpurun --timeout 600 -- bash tools/gpu_pmc_cvlr_traffic.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-cvlr_traffic}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o run --output-format csv -- python tools/cvlr_only.py > /dev/null 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/write -o run --output-format csv -- python tools/cvlr_only.py > /dev/null 2>&1 && \
python - "$O" <<'PY'
import collections, csv, os, sys
o = sys.argv[1]
per = collections.defaultdict(lambda: collections.defaultdict(float))
for name in ("fetch", "write"):
    for root, _, files in os.walk(os.path.join(o, name)):
        for f in files:
            if f.endswith("counter_collection.csv"):
                for r in csv.DictReader(open(os.path.join(root, f))):
                    if "cvlr_dma_kernel" in r["Kernel_Name"]:
                        per[r["Counter_Name"]][r.get("Dispatch_Id", "")] += float(r["Counter_Value"])
f = sorted(per["FETCH_SIZE"].values()); w = sorted(per["WRITE_SIZE"].values())
fb, wb = f[len(f) // 2] * 1024 * 2, w[len(w) // 2] * 1024
print(f"cvlr_dma_kernel 1024^2x192: fetch {fb / 1e9:.3f} GB (FETCH_SIZE x 2), write {wb / 1e9:.3f} GB, "
      f"traffic {(fb + wb) / 1e9:.3f} GB per launch vs 2.147 GB algorithmic ({len(f)} dispatches)")
PY
