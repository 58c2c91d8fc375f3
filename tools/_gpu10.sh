set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/trace -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/pmc/trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc/p1 -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/pmc/p1.log 2>&1 || echo p1 failed
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc/p2 -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/pmc/p2.log 2>&1 || echo p2 failed
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/pmc/p3.log 2>&1 || echo p3 failed
ls -R gpurun_out/pmc | head -40
