set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -s -k "tower" > gpurun_out/gpu_tests_4.log 2>&1; rc=$?
grep -E "tower max|passed|failed|Error" gpurun_out/gpu_tests_4.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tower-precision bf16x6 > gpurun_out/bench_x6.json 2> gpurun_out/bench_x6.err && cat gpurun_out/bench_x6.json
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --tower-precision fp32 > gpurun_out/bench_f32.json 2> gpurun_out/bench_f32.err && cat gpurun_out/bench_f32.json
