set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --workload c3 --steps 3 --warmup 1 > gpurun_out/b25_c3.json 2>&1; rc=$?; tail -1 gpurun_out/b25_c3.json; exit $rc
