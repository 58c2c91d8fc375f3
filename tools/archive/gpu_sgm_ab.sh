# SGM A/B (tools/_var/libsde_sgm_*.so, tools/sgm_variants.py) and the SGM GPU tests on the default build.
# usage: gpurun --timeout 600 -- bash tools/gpu_sgm_ab.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-sgm_ab}; mkdir -p $O
timeout -k 10 240 python -u tools/sgm_variants.py 1024 1024 192 > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -rf -k "sgm or SGM or config or wta" --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
