# A/B timing of tools/_var/libsde_*.so against libsde.so (tools/tower_variants.py, or the script given).
# usage: gpurun --timeout 600 -- bash tools/gpu_variants.sh TAG [script.py [args...]]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-var}; mkdir -p $O
S=${2:-tools/tower_variants.py}
shift 2 2>/dev/null || shift $#
timeout -k 10 500 python -u $S "${@:-1024}" > $O/variants.txt 2>&1 || { tail -20 $O/variants.txt; exit 1; }
grep -E "us |clock|identical|ms " $O/variants.txt | tail -60
echo done
