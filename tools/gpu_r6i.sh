set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6i}; mkdir -p $O
timeout -k 10 300 python -u tools/tower_phase.py tools/_var/libsde_phase*.so > $O/phase.txt 2>&1 || { tail -20 $O/phase.txt; exit 1; }
grep -v amdgpu.ids $O/phase.txt
SDE_VAR_GLOB='libsde_t_*.so' timeout -k 10 400 python -u tools/tower_variants.py 1024 > $O/variants.txt 2>&1 || { tail -20 $O/variants.txt; exit 1; }
grep -E "layer3 f16x3  |pair f16x3 |identical" $O/variants.txt
