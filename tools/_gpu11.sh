set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -s -k "certified or shards or golden_fused" > gpurun_out/gpu_tests_11.log 2>&1; rc=$?
grep -E "fix-up|passed|failed" gpurun_out/gpu_tests_11.log | tail -3
[ $rc -eq 0 ] || { tail -30 gpurun_out/gpu_tests_11.log; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/prof11.log 2>&1 && cat gpurun_out/prof11.log | tail -2 && cut -c1-160 gpurun_out/prof11/run_kernel_stats.csv
