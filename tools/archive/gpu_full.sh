# Full GPU check: parity tests, default bench (with CPU baseline), SGM-path bench, rocprof stats.
# usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_full.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-run}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -1 $O/bench_north_star.json
timeout -k 10 300 python bench.py --workload north_star_sgm --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_north_star_sgm.json 2> $O/bench_sgm.err || { tail -20 $O/bench_sgm.err; exit 1; }
tail -1 $O/bench_north_star_sgm.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
find $O/prof -name '*kernel_stats.csv' | head -3
