# PMC summary of the SGM scan kernels (pair, 7 launches).  usage: gpurun --timeout 600 -- bash tools/gpu_pmc_sgm.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_sgm}
mkdir -p $O
timeout -k 10 300 python tools/pmc_kernel.py run $O/p -- python tools/sgm_only.py 3 && \
python tools/pmc_kernel.py sum $O/p "sgm_scan_kernel" > $O/sgm.txt && cat $O/sgm.txt
