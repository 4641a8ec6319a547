# SQ counter passes over a kernel micro-bench (one rocprofv3 --pmc pass per set)
# usage: bash scripts/pmc_kernel.sh TAG <python args...>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=$1; shift
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY -d gpurun_out/${TAG}_p1 -o run --output-format csv -- python "$@" > gpurun_out/${TAG}_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM SQ_WAVES -d gpurun_out/${TAG}_p2 -o run --output-format csv -- python "$@" > gpurun_out/${TAG}_p2.log 2>&1
