# Round-4 PMC summaries: the tower's 64->64 layer kernel, the left-volume sweep, the CBCA passes
# (sde_cbca_lr), and HBM traffic per launch (FETCH_SIZE / WRITE_SIZE passes) of every north-star kernel.
# usage: gpurun --timeout 900 -- bash tools/gpu_pmc_r04.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r04}
mkdir -p $O
timeout -k 10 300 python tools/pmc_kernel.py run $O/tower -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
python tools/pmc_kernel.py sum $O/tower "x6p_kernel<false, false, true, true, true>" > $O/pmc_tower_layer3.txt && \
cat $O/pmc_tower_layer3.txt && \
timeout -k 10 300 python tools/pmc_kernel.py run $O/cvlr -- python tools/cvlr_only.py 1024 1024 192 left && \
python tools/pmc_kernel.py sum $O/cvlr "cvlr3" > $O/pmc_cvlr3_left.txt && cat $O/pmc_cvlr3_left.txt && \
timeout -k 10 300 python tools/pmc_kernel.py run $O/cbca -- python tools/cbca_only.py 1024 1024 192 14 2 3 && \
python tools/pmc_kernel.py sum $O/cbca "cbca_" > $O/pmc_cbca.txt && cat $O/pmc_cbca.txt && \
timeout -k 10 300 python tools/pmc_traffic_kernels.py run $O/traffic && \
python tools/pmc_traffic_kernels.py sum $O/traffic $O/traffic.json > /dev/null && cat $O/traffic.json
