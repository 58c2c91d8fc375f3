set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc22
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_VALU_MFMA_BUSY_CYCLES -d gpurun_out/pmc22/a -o run --output-format csv -- python tools/tower_only.py 1024 1024 2 > gpurun_out/pmc22/a.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_BUSY_CYCLES -d gpurun_out/pmc22/b -o run --output-format csv -- python tools/tower_only.py 1024 1024 2 > gpurun_out/pmc22/b.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_IFETCH SQ_WAVES -d gpurun_out/pmc22/c -o run --output-format csv -- python tools/tower_only.py 1024 1024 2 > gpurun_out/pmc22/c.log 2>&1
ls gpurun_out/pmc22
