# attention micro-bench PMC counters (two passes; no tracing domains besides kernel-trace)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/kpmc1 -o run --output-format csv -- python scripts/kbench.py attn --batch 16 --iters 1 > gpurun_out/kpmc1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_INSTS_SALU -d gpurun_out/kpmc2 -o run --output-format csv -- python scripts/kbench.py attn --batch 16 --iters 1 > gpurun_out/kpmc2.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY -d gpurun_out/kpmc3 -o run --output-format csv -- python scripts/kbench.py attn --batch 16 --iters 1 > gpurun_out/kpmc3.log 2>&1
