# round 5 / aa: persistent GEMM form at long K with nt output stores: SM_GEMM_PP_MAXK (default 128) x
# SM_GEMM_PP_ROUNDS (tiles per block; 0 = one resident round of persistent blocks), kbench gemm, one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { echo "== $1"; (export $2; timeout -k 10 300 python scripts/kbench.py gemm --iters 5) || exit 1; }
for pass in 1 2; do
  run "default (pp K<=128)" "SM_GEMM_PP_MAXK=128"
  run "pp K<=1536, persistent" "SM_GEMM_PP_MAXK=1536"
  run "pp K<=1536, 2 tiles/block" "SM_GEMM_PP_MAXK=1536 SM_GEMM_PP_ROUNDS=2"
  run "pp K<=1536, 4 tiles/block" "SM_GEMM_PP_MAXK=1536 SM_GEMM_PP_ROUNDS=4"
  run "pp K<=1536, 8 tiles/block" "SM_GEMM_PP_MAXK=1536 SM_GEMM_PP_ROUNDS=8"
done > gpurun_out/r05aa_gemm_pp.txt 2>&1
cat gpurun_out/r05aa_gemm_pp.txt
