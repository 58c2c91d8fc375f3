set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc17
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_WAVES -d gpurun_out/pmc17/a -o run --output-format csv -- python tools/cbca_only.py 1024 1024 192 14 2 > gpurun_out/pmc17/a.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE TCC_HIT_sum -d gpurun_out/pmc17/b -o run --output-format csv -- python tools/cbca_only.py 1024 1024 192 14 2 > gpurun_out/pmc17/b.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_MISS_sum -d gpurun_out/pmc17/c -o run --output-format csv -- python tools/cbca_only.py 1024 1024 192 14 2 > gpurun_out/pmc17/c.log 2>&1
ls gpurun_out/pmc17/*/
