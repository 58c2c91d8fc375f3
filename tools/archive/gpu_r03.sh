# Round-3 check: every -m gpu test, the default bench line (with CPU baselines), rocprofv3 kernel
# stats of the north_star and north_star_sgm workloads, and PMC HBM traffic per kernel.
# usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_r03.sh TAG [skip-tests]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -c 600 $O/bench_north_star.json
for w in north_star north_star_sgm; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench_$w.json 2> $O/prof_$w.err || { tail -20 $O/prof_$w.err; exit 1; }
done
timeout -k 10 300 python tools/pmc_traffic_kernels.py run $O/pmc_traffic && python tools/pmc_traffic_kernels.py sum $O/pmc_traffic $O/traffic.json > /dev/null
echo done
