set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6r}; mkdir -p $O
SDE_VAR_GLOB='libsde_t_*.so' timeout -k 10 400 python -u tools/tower_variants.py 1024 > $O/variants.txt 2>&1 || { tail -20 $O/variants.txt; exit 1; }
grep -E "layer3 f16x3  |layer3 f16x3 split|pair f16x3 |identical" $O/variants.txt
