# Round-3 final check: every -m gpu test, smoke(), the default bench line (CPU baselines included), the
# north_star_sgm / c3 / cones bench lines, rocprofv3 kernel stats of north_star and north_star_sgm,
# and PMC HBM traffic per kernel.  usage: gpurun --timeout 1100 -- bash tools/gpu_r03_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03final}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -c 300 $O/bench_north_star.json
for w in north_star_sgm c3 cones; do
  timeout -k 10 300 python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
done
for w in north_star north_star_sgm; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$w -o run --output-format csv -- python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_bench_$w.json 2> $O/prof_$w.err || { tail -20 $O/prof_$w.err; exit 1; }
done
timeout -k 10 300 python tools/pmc_traffic_kernels.py run $O/pmc_traffic && python tools/pmc_traffic_kernels.py sum $O/pmc_traffic $O/traffic.json > /dev/null
timeout -k 10 300 python tools/pmc_kernel.py run $O/cv -- python tools/cv_only.py 1024 1024 192 certified && \
python tools/pmc_kernel.py sum $O/cv "cv_wta_row2" > $O/pmc_cv_wta_row2.txt
echo done
