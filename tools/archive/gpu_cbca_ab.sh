# CBCA A/B (tools/lib_variants.py cbca: in-tree lib vs tools/_var variants).  usage: gpurun -- bash tools/gpu_cbca_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-cbca_ab}; mkdir -p $O
timeout -k 10 240 python -u tools/lib_variants.py cbca > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
