set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -k "sgm or post or matcher or disparity" > gpurun_out/gpu_tests_14.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_14.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/gpu_tests_14.log | head -20; exit $rc; }
timeout -k 10 300 python tools/stage_timing.py 1024 1024 192 > gpurun_out/stage14.json 2>&1; rc=$?; cat gpurun_out/stage14.json | tail -2; exit $rc
