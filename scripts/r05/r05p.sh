# round 5 / p: SQ counters before / after for this round's GEMM-family changes:
#   the statistics epilogue (base = the library before it, ab_lib/libsslmae_base.so) on kbench bnstats,
#   the persistent small-K form (SM_GEMM_PP=0 / 1) on the stage-0 expand GEMM (kbench gemm --only "s0 expand").
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05p}
BASE="SM_LIB_PATH=$GRAFT_REPO_ROOT/ab_lib/libsslmae_base.so"
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY"
C2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES"
run() {   # tag, env, kbench args
  local tg=$1 ev=$2; shift 2
  env $ev timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/${T}_${tg}_p1 -o run --output-format csv -- python3 scripts/kbench.py "$@" --iters 1 > gpurun_out/${T}_${tg}_p1.log 2>&1 && \
  env $ev timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/${T}_${tg}_p2 -o run --output-format csv -- python3 scripts/kbench.py "$@" --iters 1 > gpurun_out/${T}_${tg}_p2.log 2>&1
}
run stats_base "$BASE" bnstats || exit 1
run stats_new "SM_NONE=1" bnstats || exit 1
run pp0 "SM_GEMM_PP=0" gemm --only "s0 expand" || exit 1
run pp1 "SM_GEMM_PP=1" gemm --only "s0 expand" || exit 1
timeout -s KILL 60 rocprofv3 --pmc SQ_VALU_MFMA_COEXEC_CYCLES -d gpurun_out/${T}_coexec -o run --output-format csv -- python3 scripts/kbench.py bnstats --iters 1 > gpurun_out/${T}_coexec.log 2>&1 || echo "coexec counter pass failed" >> gpurun_out/${T}_coexec.log
exit 0
