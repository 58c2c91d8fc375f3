# Quick GPU iteration: selected tests (-k expr) + rocprof kernel stats of a tool script.
# usage: gpurun -- bash tools/gpu_quick.sh TAG "pytest -k expr" "python tools/x.py args"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1; K=$2; shift 2
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "$K" -s > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
fi
i=0
for cmd in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof$i -o run --output-format csv -- $cmd > $O/cmd$i.log 2>&1 || { tail -30 $O/cmd$i.log; exit 1; }
  tail -2 $O/cmd$i.log
  python3 - "$O/prof$i" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(f"{float(r['AverageNs'])/1e3:10.1f} us x{r['Calls']:>4}  {r['Name'][:110]}")
PY
done
