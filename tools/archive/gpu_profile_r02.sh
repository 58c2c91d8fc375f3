# Round-2 profiles: rocprofv3 kernel stats of the three bench workloads (north_star, north_star_sgm,
# c3) -> gpurun_out/TAG/<workload>/ + the bench lines.
# usage: gpurun --timeout 1100 -- bash tools/gpu_profile_r02.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-prof}
O=gpurun_out/$TAG
mkdir -p $O
for w in north_star north_star_sgm c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$w -o run --output-format csv -- python bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_$w.json 2> $O/bench_$w.err || { tail -20 $O/bench_$w.err; exit 1; }
  tail -c 400 $O/bench_$w.json
done
