# Round-2 (session 3) profiles: rocprofv3 kernel stats of the three bench workloads + the default
# bench line + PMC of the L/R volume kernel.  usage: gpurun --timeout 1100 -- bash tools/gpu_profile_s3.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-prof}
O=gpurun_out/$TAG
mkdir -p $O
for w in north_star north_star_sgm c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$w -o run --output-format csv -- python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  tail -c 300 $O/bench_$w.json
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
timeout -k 10 300 python tools/pmc_kernel.py run $O/pmc_cvlr -- python tools/cvlr_only.py && \
python tools/pmc_kernel.py sum $O/pmc_cvlr "cvlr" > $O/pmc_cvlr.txt && cat $O/pmc_cvlr.txt
