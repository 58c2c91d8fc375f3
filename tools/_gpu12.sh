set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc12
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/pmc12/p1 -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/pmc12/p1.log 2>&1 || echo p1 failed
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_MFMA TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc12/p2 -o run --output-format csv -- python tools/cv_only.py 1024 1024 192 certified > gpurun_out/pmc12/p2.log 2>&1 || echo p2 failed
grep fixups gpurun_out/pmc12/p1.log
