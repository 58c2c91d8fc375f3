# Tower tests, then the tower A/B (tools/tower_variants.py) against tools/_var libraries.
# usage: gpurun --timeout 900 -- bash tools/gpu_tower_ab.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "${2:-tower}" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python tools/tower_variants.py 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
