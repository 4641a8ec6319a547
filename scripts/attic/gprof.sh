# GEMM fixed-cost sweep + PMC counters of the fwd GEMM at one shape
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python scripts/kbench.py gemmk --batch 256 > gpurun_out/kb_gemmk.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d gpurun_out/gpmc1 -o run --output-format csv -- python scripts/kbench.py gemm --batch 64 --iters 1 --only "dec qkv" > gpurun_out/gpmc1.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE -d gpurun_out/gpmc2 -o run --output-format csv -- python scripts/kbench.py gemm --batch 64 --iters 1 --only "dec qkv" > gpurun_out/gpmc2.log 2>&1
