# SQ counters (two passes) of the bf16 GEMM at three step shapes (kbench gemm: forward, dX, dW
# per shape).   usage: bash scripts/gemm_pmc.sh TAG
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-gp}
for s in "dec qkv" "dec fc1" "s0 expand"; do
  n=$(echo $s | tr ' ' '_')
  timeout -k 10 200 python scripts/kbench.py gemm --only "$s" --iters 5 > gpurun_out/${TAG}_${n}_t.txt 2>&1 || exit 1
  bash scripts/pmc_kernel.sh ${TAG}_${n} scripts/kbench.py gemm --only "$s" --iters 1 || exit 1
done
