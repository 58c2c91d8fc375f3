# PMC summary of the tower's layer 3 (both images per launch, f16x3): the Winograd kernel and the
# direct kernel.  usage: gpurun --timeout 600 -- bash tools/gpu_pmc_wino.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_wino}
mkdir -p $O
timeout -k 10 200 python tools/pmc_kernel.py run $O/w -- python tools/wino_layer.py wino 5 && \
timeout -k 10 200 python tools/pmc_kernel.py run $O/d -- python tools/wino_layer.py direct 5 && \
python tools/pmc_kernel.py sum $O/w "wino_kernel" > $O/wino.txt && \
python tools/pmc_kernel.py sum $O/d "x6p_kernel" > $O/direct.txt && cat $O/wino.txt $O/direct.txt
