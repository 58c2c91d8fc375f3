# PMC summary of the tower's middle layer (both images per launch, f16x3) and of the certified CV+WTA
# kernel: MFMA busy cycles, VALU / LDS instruction counts, waits, clock (GRBM_GUI_ACTIVE / 8 XCDs).
# usage (from this container): gpurun --timeout 900 -- bash tools/gpu_pmc_tower.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_tower}
mkdir -p $O
timeout -k 10 400 python tools/pmc_kernel.py run $O/pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
python tools/pmc_kernel.py sum $O/pmc "x6p_kernel<false, false, true, true, true>" > $O/tower_layer3.txt && \
python tools/pmc_kernel.py sum $O/pmc "cv_wta_row_kernel" > $O/cv_wta_row.txt && cat $O/tower_layer3.txt $O/cv_wta_row.txt
