set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c3b; mkdir -p $O
timeout -k 10 200 python tools/lib_variants.py cvlr 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
timeout -k 10 300 python tools/pmc_kernel.py run $O/pmc -- python tools/cvlr_only.py && \
python tools/pmc_kernel.py sum $O/pmc "cvlr3" > $O/pmc_cvlr3.txt && cat $O/pmc_cvlr3.txt
