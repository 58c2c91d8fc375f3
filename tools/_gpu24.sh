set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/t24.log 2>&1; rc=$?
tail -2 gpurun_out/t24.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t24.log | head -20; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof24 -o run --output-format csv -- python bench.py > gpurun_out/b24_ns.json 2>&1; rc=$?; grep metric gpurun_out/b24_ns.json | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/b24_c3.json 2>&1; rc=$?; tail -1 gpurun_out/b24_c3.json | cut -c1-300; exit $rc
