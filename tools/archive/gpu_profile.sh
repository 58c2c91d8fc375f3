# Round profile refresh: full GPU check (tools/archive/gpu_full.sh) + PMC HBM traffic of the default
# workload's roofline kernel (tools/pmc_traffic.py) -> gpurun_out/TAG/.
# usage (from this container): gpurun --timeout 1100 -- bash tools/gpu_profile.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-prof}
bash tools/archive/gpu_full.sh $TAG || exit 1
cp profiles/r01/traffic.json gpurun_out/$TAG/traffic.json
timeout -k 10 400 python tools/pmc_traffic.py run north_star gpurun_out/$TAG/pmc && \
python tools/pmc_traffic.py sum north_star gpurun_out/$TAG/pmc gpurun_out/$TAG/traffic.json
