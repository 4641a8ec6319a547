# round 5 / ac: persistent GEMM form at N = 384 (SM_GEMM_PP_MINN) and K up to 1536 (SM_GEMM_PP_MAXK), kbench gemm, one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { echo "== $1"; (export $2; timeout -k 10 300 python scripts/kbench.py gemm --iters 5) || exit 1; }
for pass in 1 2; do
  run "default (K<=128 | K<=384 & N>=512)" "SM_GEMM_PP_MINN=512"
  run "N>=384" "SM_GEMM_PP_MINN=384"
  run "N>=384, K<=1536" "SM_GEMM_PP_MINN=384 SM_GEMM_PP_MAXK=1536"
done > gpurun_out/r05ac_gemm_pp_n384.txt 2>&1
cat gpurun_out/r05ac_gemm_pp_n384.txt
