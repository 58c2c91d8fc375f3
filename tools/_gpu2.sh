set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_ns.json 2> gpurun_out/bench_ns.err || { echo "bench failed"; tail -20 gpurun_out/bench_ns.err; exit 1; }
cat gpurun_out/bench_ns.json
timeout -k 10 200 python bench.py --workload cones --no-cpu-baseline > gpurun_out/bench_cones.json 2>&1 && cat gpurun_out/bench_cones.json
timeout -k 10 200 python bench.py --workload cv --no-cpu-baseline > gpurun_out/bench_cv.json 2>&1 && cat gpurun_out/bench_cv.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_bench.json 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_bench.json; exit 1; }
timeout -k 10 300 python tools/stage_timing.py > gpurun_out/stage_timing.json 2>&1; cat gpurun_out/stage_timing.json
find gpurun_out/prof_r1 -name '*stats*'
