set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c3a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -k "hwd_volumes or cvlr or disparity_compute" > $O/tests.log 2>&1; rc=$?; tail -5 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/lib_variants.py cvlr 2>&1 | tee $O/ab.log
