set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/gpu_tests_3.log 2>&1; rc=$?
tail -15 gpurun_out/gpu_tests_3.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_ns3.json 2> gpurun_out/bench_ns3.err && cat gpurun_out/bench_ns3.json
