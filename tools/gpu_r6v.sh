# CV fix-up rewrite check: the certified / exact CV+WTA GPU tests, C5 bench, rocprof of the north-star bench
# (fix-up kernel time).  usage: gpurun --timeout 900 -- bash tools/gpu_r6v.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6v}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -rf -s --timeout 600 --timeout-method thread -k "certified or config5 or cv_wta or shard or multirank or fixup or tie" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed|fix-up" $O/tests.log | tail -5
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); st=d['stages']; print('c5', d['ms_per_step'], st['cv_wta_ms'], st['cv_exact_fixup_pixels'], st['tower_ms_pair'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-c3 > $O/prof_bench.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_c5.json 2> $O/prof_c5.err || { tail -20 $O/prof_c5.err; exit 1; }
python - "$O" <<'PY'
import csv, sys
for f in ("prof", "prof_c5"):
    for r in csv.DictReader(open(f"{sys.argv[1]}/{f}/run_kernel_stats.csv")):
        if any(k in r["Name"] for k in ("fixup", "row2", "argmin_chunks")):
            print(f, r["Name"][:60], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
echo done
