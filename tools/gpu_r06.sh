# Quick round-6 check: every -m gpu test, smoke(), the default bench line, a rocprofv3 kernel-stats run
# of the north-star bench, and tools/tower_variants.py over tools/_var.  usage: gpurun --timeout 1100 -- bash tools/gpu_quick5.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6}; mkdir -p $O
if [ "$2" != "skip-tests" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -c 400 $O/bench_north_star.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_north_star -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3 > $O/prof_bench_north_star.json 2> $O/prof_north_star.err || { tail -20 $O/prof_north_star.err; exit 1; }
if ls tools/_var/libsde_*.so > /dev/null 2>&1; then
  timeout -k 10 300 python tools/tower_variants.py 1024 > $O/tower_variants.txt 2>&1 || { tail -20 $O/tower_variants.txt; exit 1; }
  grep -E "us |clock" $O/tower_variants.txt | tail -24
fi
echo done
