# L/R volume A/B (tools/lib_variants.py cvlr: in-tree lib vs tools/_var variants) + the L/R volume GPU tests.
# usage: gpurun --timeout 600 -- bash tools/gpu_cvlr_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-cvlr_ab}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf -k "hwd or cvlr or config or golden" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 240 python -u tools/lib_variants.py cvlr > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
grep -v amdgpu.ids $O/ab.log
