# Round-5 PMC summaries: the tower's middle layer and layer 2 on the 16x16x32 kernel (both images per launch, f16x3) and
# the certified CV+WTA kernel (tools/pmc_kernel.py: one --pmc pass per counter group).
# usage (from this container): gpurun --timeout 900 -- bash tools/gpu_pmc_r05.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r05}
mkdir -p $O
timeout -k 10 500 python tools/pmc_kernel.py run $O/pmc -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline && \
python tools/pmc_kernel.py sum $O/pmc "conv64_h16_kernel<false, true, true, false, false, false, false>" > $O/tower_layer3.txt && \
python tools/pmc_kernel.py sum $O/pmc "conv64_h16_kernel<false, false, true, false, false, false, true>" > $O/tower_layer2.txt && \
python tools/pmc_kernel.py sum $O/pmc "cv_wta_row2_kernel" > $O/cv_wta_row2.txt && cat $O/tower_layer3.txt $O/tower_layer2.txt $O/cv_wta_row2.txt
