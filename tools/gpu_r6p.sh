set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6p}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf -s --timeout 600 --timeout-method thread -k "certified or config5 or cv_wta or shard or multirank" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|fix-up" $O/tests.log | tail -5
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); st=d['stages']; print('c5', d['ms_per_step'], st['cv_wta_ms'], st['cv_exact_fixup_pixels'], st['tower_ms_pair'])"
