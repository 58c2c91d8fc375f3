# Round-3 PMC summaries of the current L/R volume kernel, certified CV+WTA row kernel and SGM pair.
# usage: gpurun --timeout 900 -- bash tools/gpu_pmc_r03.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmc_r03}
mkdir -p $O
timeout -k 10 300 python tools/pmc_kernel.py run $O/cvlr -- python tools/cvlr_only.py && \
python tools/pmc_kernel.py sum $O/cvlr "cvlr3" > $O/pmc_cvlr3.txt && cat $O/pmc_cvlr3.txt && \
timeout -k 10 300 python tools/pmc_kernel.py run $O/cv -- python tools/cv_only.py 1024 1024 192 certified && \
python tools/pmc_kernel.py sum $O/cv "cv_wta_row2" > $O/pmc_cv_wta_row2.txt && cat $O/pmc_cv_wta_row2.txt && \
timeout -k 10 300 python tools/pmc_kernel.py run $O/sgm -- python tools/sgm_only.py 3 && \
python tools/pmc_kernel.py sum $O/sgm "sgm_scan_kernel" > $O/pmc_sgm_pair.txt && cat $O/pmc_sgm_pair.txt
