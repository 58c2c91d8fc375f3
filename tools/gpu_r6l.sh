set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6l}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf -s --timeout 600 --timeout-method thread -k "certified or config5 or tower or cv_wta" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|fix-up" $O/tests.log | tail -5
SDE_VAR_GLOB='libsde_t_*.so' timeout -k 10 400 python -u tools/tower_variants.py 1024 > $O/variants.txt 2>&1 || { tail -20 $O/variants.txt; exit 1; }
grep -E "layer3 f16x3  |pair f16x3 |identical" $O/variants.txt
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); st=d['stages']; print('c5', d['ms_per_step'], st['cv_wta_ms'], st['cv_exact_fixup_pixels'], st['tower_ms_pair'])"
