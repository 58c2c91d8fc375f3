set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -s -k "certified or shards or golden_fused" > gpurun_out/gpu_tests_5.log 2>&1; rc=$?
grep -E "fix-up|passed|failed|Error|assert" gpurun_out/gpu_tests_5.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cert.json 2> gpurun_out/bench_cert.err && cat gpurun_out/bench_cert.json
timeout -k 10 300 python bench.py --workload cv --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cv_cert.json 2> gpurun_out/bench_cv_cert.err && cat gpurun_out/bench_cv_cert.json
