# HBM-side traffic and L2 hit rate of a kernel micro-bench (separate rocprofv3 --pmc passes)
# usage: bash scripts/pmc_l2.sh TAG <python args...>
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=$1; shift
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${TAG}_p1 -o run --output-format csv -- python "$@" > gpurun_out/${TAG}_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/${TAG}_p2 -o run --output-format csv -- python "$@" > gpurun_out/${TAG}_p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${TAG}_p3 -o run --output-format csv -- python "$@" > gpurun_out/${TAG}_p3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_INSTS_LDS -d gpurun_out/${TAG}_p4 -o run --output-format csv -- python "$@" > gpurun_out/${TAG}_p4.log 2>&1
python scripts/pmc_sum.py gpurun_out/${TAG} > gpurun_out/${TAG}_summary.txt
