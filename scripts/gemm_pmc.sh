# PMC counters of the GEMM kernels on the bench shapes (kbench gemm), one pass per counter set
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ONLY=${1:-dec qkv}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY -d gpurun_out/gpmc1 -o run --output-format csv -- python scripts/kbench.py gemm --iters 1 --only "$ONLY" > gpurun_out/gpmc1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_CYCLES -d gpurun_out/gpmc2 -o run --output-format csv -- python scripts/kbench.py gemm --iters 1 --only "$ONLY" > gpurun_out/gpmc2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum -d gpurun_out/gpmc3 -o run --output-format csv -- python scripts/kbench.py gemm --iters 1 --only "$ONLY" > gpurun_out/gpmc3.log 2>&1
