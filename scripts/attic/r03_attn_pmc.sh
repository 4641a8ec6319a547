# SQ counters of the attention kernels (kbench attn, B=32), two --pmc passes
set -e
TAG=${1:-r03h}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY -d gpurun_out/${TAG}_p1 -o run --output-format csv -- python scripts/kbench.py attn --batch 32 --drop 0.1 --iters 1 > gpurun_out/${TAG}_p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAVES GRBM_GUI_ACTIVE -d gpurun_out/${TAG}_p2 -o run --output-format csv -- python scripts/kbench.py attn --batch 32 --drop 0.1 --iters 1 > gpurun_out/${TAG}_p2.log 2>&1
python scripts/pmc_sum.py gpurun_out/${TAG} attn > gpurun_out/${TAG}_sum.txt
