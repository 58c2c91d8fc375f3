# Round-6 full check + evidence: every -m gpu test, smoke(), the default bench line, a rocprofv3 kernel-stats run of
# the north-star bench (no C3 stage, so the tower/CV launches are the north star's only), PMC HBM traffic per launch
# of the north-star kernels (profiles/r06/traffic.json), PMC counter groups of the tower's layer 3 and the
# certified CV+WTA.  usage: gpurun --timeout 1200 -- bash tools/gpu_r06_final.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6f}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -c 300 $O/bench_north_star.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_north_star -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3 > $O/prof_bench_north_star.json 2> $O/prof_north_star.err || { tail -20 $O/prof_north_star.err; exit 1; }
timeout -k 10 400 python tools/pmc_traffic_kernels.py run $O/traffic > $O/traffic_run.log 2>&1 || { tail -20 $O/traffic_run.log; exit 1; }
python tools/pmc_traffic_kernels.py sum $O/traffic $O/traffic.json > /dev/null || exit 1
timeout -k 10 400 python tools/pmc_kernel.py run $O/pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c3 || exit 1
python tools/pmc_kernel.py sum $O/pmc "conv64_h16_kernel<false, true, true, false, false, false, false>" > $O/pmc_tower_layer3.txt || exit 1
python tools/pmc_kernel.py sum $O/pmc "cv_wta_row2_kernel" > $O/pmc_cv_wta_row2.txt || exit 1
echo done
