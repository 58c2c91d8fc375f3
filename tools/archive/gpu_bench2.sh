# Two default bench runs back to back (run-to-run spread of the driver's line).  usage: gpurun -- bash tools/gpu_bench2.sh TAG
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-bench2}; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python bench.py > $O/bench_$i.json 2> $O/bench_$i.err || { tail -20 $O/bench_$i.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['steps'],d['stages']['reference_gpu_path']['cv_aggregation_aggregate']['hbm_frac'])"
done
