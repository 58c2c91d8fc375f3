set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -k "certified or shards or golden_fused" > gpurun_out/gpu_tests_6.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests_6.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cv6 -o run --output-format csv -- python bench.py --workload cv --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_cv6.json 2>&1 && cat gpurun_out/prof_cv6/run_kernel_stats.csv | cut -c1-200
