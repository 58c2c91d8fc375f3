set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -k "cbca or sgm" > gpurun_out/gpu_tests_15.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_15.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_15.log | head -20; exit $rc; }
timeout -k 10 300 python tools/stage_timing.py 1024 1024 192 > gpurun_out/stage15.json 2>&1; rc=$?; tail -1 gpurun_out/stage15.json; exit $rc
