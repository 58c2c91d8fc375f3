set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r6k}; mkdir -p $O
timeout -k 10 300 python bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
tail -c 300 $O/bench_c5.json
timeout -k 10 600 python -u tools/sgm_skew_probe.py 10 > $O/sgm_skew.txt 2>&1 || { tail -20 $O/sgm_skew.txt; exit 1; }
grep -v amdgpu.ids $O/sgm_skew.txt
