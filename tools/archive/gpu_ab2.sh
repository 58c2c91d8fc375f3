# SGM / CBCA tests, then the certified CV+WTA diagnostic builds and the SGM A/B (tools/_var).
# usage: gpurun --timeout 900 -- bash tools/gpu_ab2.sh TAG [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread -k "${2:-sgm}" > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
CV_ROUNDS=${CV_ROUNDS:-5} timeout -k 10 300 python tools/cv_variants.py 2>&1 | grep -v amdgpu.ids | tee $O/cv.log
[ -n "$3" ] && timeout -k 10 300 python tools/lib_variants.py sgm 2>&1 | grep -v amdgpu.ids | tee $O/ab.log
