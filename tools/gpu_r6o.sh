set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6o}; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/prof_bench_c5.json 2> $O/prof_c5.err || { tail -20 $O/prof_c5.err; exit 1; }
python - <<PY
import csv, statistics, collections
d=collections.defaultdict(list)
for r in csv.DictReader(open('$O/prof_c5/run_kernel_trace.csv')):
    n=r['Kernel_Name']; dur=(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3
    d[n[:70]].append(dur)
for k,v in sorted(d.items(), key=lambda kv: -sum(kv[1])): print(f"{k:70s} n={len(v)} med={statistics.median(v):9.1f} us")
PY
