set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out profiles/r01
timeout -k 10 300 python bench.py --workload north_star_sgm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b23_nss.json 2>&1; rc=$?; tail -1 gpurun_out/b23_nss.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/pmc_traffic.py run north_star gpurun_out/pmc23 && python tools/pmc_traffic.py sum north_star gpurun_out/pmc23 gpurun_out/traffic.json
