# Every -m gpu test, then the A/B timing of tools/_var variants (tools/lib_variants.py WHAT).
# usage: gpurun --timeout 1100 -- bash tools/gpu_full_ab.sh TAG WHAT
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/tests.log | head -20; exit $rc; }
[ -n "$2" ] && timeout -k 10 300 python tools/lib_variants.py $2 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
exit 0
