# A/B of tools/_var/libsde_*.so against the in-tree library (tools/lib_variants.py WHAT), optional -k tests first.
# usage: gpurun -- bash tools/gpu_ab.sh TAG WHAT [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
if [ -n "$3" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "$3" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 300 python tools/lib_variants.py $2 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
