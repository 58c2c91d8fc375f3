# cvlr A/B: the cvlr parity tests, then tools/lib_variants.py cvlr (in-tree library vs tools/_var/*.so).
# usage: gpurun --timeout 600 -- bash tools/gpu_cvlr.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "hwd or cvlr or config4 or config3 or sgm_path" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u tools/lib_variants.py cvlr > $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
cat $O/ab.log
