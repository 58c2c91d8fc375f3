set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests -m gpu -q -k cbca > gpurun_out/t16.log 2>&1; tail -1 gpurun_out/t16.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof16 -o run --output-format csv -- python tools/cbca_only.py 1024 1024 192 14 > gpurun_out/p16.log 2>&1 && cut -c1-150 gpurun_out/prof16/run_kernel_stats.csv | grep cbca
