set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -s > gpurun_out/gpu_tests_13.log 2>&1; rc=$?
grep -E "fix-up|tower max|passed|failed" gpurun_out/gpu_tests_13.log | tail -4
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_13.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof13 -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench13.json 2>&1 && grep metric gpurun_out/bench13.json && cut -c1-150 gpurun_out/prof13/run_kernel_stats.csv
