# round 5 / ai: SQ counters before / after for the persistent GEMM form at K = 384: the decoder
# qkv forward (kbench gemm --only "dec qkv") as one-tile-per-block v2 (SM_GEMM_PP_MINN=100000) and as gemm_bf16_pp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05ai}
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY"
C2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES"
run() {   # tag, env, kbench args
  local tg=$1 ev=$2; shift 2
  env $ev timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/${T}_${tg}_p1 -o run --output-format csv -- python3 scripts/kbench.py "$@" --iters 1 > gpurun_out/${T}_${tg}_p1.log 2>&1 && \
  env $ev timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/${T}_${tg}_p2 -o run --output-format csv -- python3 scripts/kbench.py "$@" --iters 1 > gpurun_out/${T}_${tg}_p2.log 2>&1 && \
  env $ev timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES -d gpurun_out/${T}_${tg}_p3 -o run --output-format csv -- python3 scripts/kbench.py "$@" --iters 1 > gpurun_out/${T}_${tg}_p3.log 2>&1
}
run v2 "SM_GEMM_PP_MINN=100000" gemm --only "dec qkv" || exit 1
run pp "SM_GEMM_PP_MINN=512" gemm --only "dec qkv" || exit 1
python3 scripts/pmc_ab_table.py gpurun_out/${T}_v2 gpurun_out/${T}_pp "gemm_bf16_v2<true, true||gemm_bf16_pp<true, 0>" v2 pp
