# cvlr diagnostics: A/B of tools/_var variants (lib_variants.py cvlr), then PMC of the in-tree kernel.
# usage: gpurun --timeout 600 -- bash tools/gpu_cvlr_diag.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python -u tools/lib_variants.py cvlr > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 300 python tools/pmc_kernel.py run $O/p -- python tools/cvlr_only.py && \
python tools/pmc_kernel.py sum $O/p "cvlr" > $O/pmc.txt && cat $O/pmc.txt
