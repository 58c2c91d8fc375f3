# Round-3 session-3 check after the container re-creation: every -m gpu test, smoke(), the default bench line.
# usage: gpurun --timeout 900 -- bash tools/gpu_r03c.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03c}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -c 400 $O/bench_north_star.json
echo done
