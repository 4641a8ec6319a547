# GEMM tile-variant probe: kbench gemm + gemmw at the default variant choice, BM = 256 and BM = 128
set -e
TAG=${1:-r03g2}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in 0 2 3; do
SM_GEMM_VARIANT=$v timeout -k 10 300 python scripts/kbench.py gemm --iters 5 > gpurun_out/${TAG}_gemm_v$v.log 2>&1
SM_GEMM_VARIANT=$v timeout -k 10 300 python scripts/kbench.py gemmw --iters 5 > gpurun_out/${TAG}_gemmw_v$v.log 2>&1
done
