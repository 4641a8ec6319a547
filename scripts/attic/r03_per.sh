# persistent forward GEMM: GEMM tests, then kbench gemm / gemmw with the persistent form off and on
set -e
TAG=${1:-r03p2}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "gemm or linear" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
SM_GEMM_PER=0 timeout -k 10 300 python scripts/kbench.py gemmw --iters 5 > gpurun_out/${TAG}_w_off$i.log 2>&1
timeout -k 10 300 python scripts/kbench.py gemmw --iters 5 > gpurun_out/${TAG}_w_on$i.log 2>&1
done
SM_GEMM_PER=0 timeout -k 10 300 python scripts/kbench.py gemm --iters 5 --only s0 > gpurun_out/${TAG}_g_off.log 2>&1
timeout -k 10 300 python scripts/kbench.py gemm --iters 5 --only s0 > gpurun_out/${TAG}_g_on.log 2>&1
