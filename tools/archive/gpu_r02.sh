# Round-2 GPU check: every -m gpu test (verbose, the config-size tests print progress), then the
# default bench line (parity checks + the reference GPU path stages) and its rocprof stats.
# usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_r02.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
K=${2:-}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -rf --timeout 900 --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -3 $O/tests.log
grep -E "PASSED|FAILED" $O/tests.log | grep -E "config|row_band" || true
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -1 $O/bench_north_star.json
