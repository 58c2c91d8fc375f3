# Every -m gpu test, the default bench line, and the SGM pair's PMC (LDS bank conflicts of the fused WTA).
# usage: gpurun --timeout 900 -- bash tools/gpu_r03b.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03b}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py > $O/bench_north_star.json 2> $O/bench_north_star.err || { tail -20 $O/bench_north_star.err; exit 1; }
tail -c 300 $O/bench_north_star.json
timeout -k 10 300 python tools/pmc_kernel.py run $O/sgm -- python tools/sgm_only.py 3 && \
python tools/pmc_kernel.py sum $O/sgm "sgm_scan_kernel" > $O/pmc_sgm_pair.txt && grep -A25 "192, 7, true" $O/pmc_sgm_pair.txt | grep -E "LDS|WAVE_CYCLES"
