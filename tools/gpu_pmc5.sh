# Round-5 PMC: HBM traffic per launch of the north star's dominant kernel (profiles/r05/traffic.json via
# tools/pmc_traffic.py, two separate --pmc passes) and a counter pass over the tower's layer 3.
# usage: gpurun --timeout 900 -- bash tools/gpu_pmc5.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pm5}; mkdir -p $O
timeout -k 10 400 python tools/pmc_traffic.py run north_star $O/traffic > $O/traffic_run.log 2>&1 || { tail -20 $O/traffic_run.log; exit 1; }
python tools/pmc_traffic.py sum north_star $O/traffic $O/traffic.json || exit 1
echo done
