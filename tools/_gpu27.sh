set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/t27.log 2>&1; rc=$?
tail -2 gpurun_out/t27.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/t27.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload north_star_sgm --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/b27.json 2>&1; rc=$?; tail -1 gpurun_out/b27.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['stages'])"; exit $rc
