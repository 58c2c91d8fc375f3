set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -s -k "tower or matcher or split" > gpurun_out/t19.log 2>&1; rc=$?
grep -E "tower max|passed|failed" gpurun_out/t19.log | tail -3
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t19.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof19 -o run --output-format csv -- python tools/tower_only.py 1024 1024 3 > gpurun_out/p19.log 2>&1 && cut -d, -f1-4 gpurun_out/prof19/run_kernel_stats.csv | cut -c1-40,150-
