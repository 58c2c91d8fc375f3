# Preprocess check: its GPU tests, the bench line, and a rocprofv3 kernel-stats run of the bench.
# usage: gpurun --timeout 900 -- bash tools/gpu_pp.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-pp1}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "preprocess or tower_forward_batch or matcher" --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));s=d['stages'];print(d['value'],d['ms_per_step'],s['tower_ms_pair'],s['cv_wta_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/prof.json 2> $O/prof.err; echo "rocprof exit $?"
grep -E "preprocess|np_|znorm|absmax" $O/prof/run_kernel_stats.csv | cut -c1-160
echo done
