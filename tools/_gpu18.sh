set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc18
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc18/a -o run --output-format csv -- python tools/tower_only.py 1024 1024 2 > gpurun_out/pmc18/a.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc18/b -o run --output-format csv -- python tools/tower_only.py 1024 1024 2 > gpurun_out/pmc18/b.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc18/c -o run --output-format csv -- python tools/tower_only.py 1024 1024 3 > gpurun_out/pmc18/c.log 2>&1 && cut -c1-160 gpurun_out/pmc18/c/run_kernel_stats.csv
