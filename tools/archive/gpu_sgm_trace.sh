set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
O=gpurun_out/sgmprof; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python bench.py --workload north_star_sgm --steps 2 --warmup 1 --no-cpu-baseline > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
echo done
