# 128-row waves (4 waves per 256 x 128 tile, SM_GEMM_WM=128) against the 8-wave v2 GEMM:
# GEMM tests under the knob, then kbench gemm alternating (same box, same build).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04n}
SM_GEMM_WM=128 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "gemm or linear" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  timeout -k 10 300 python scripts/kbench.py gemm --iters 10 > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  SM_GEMM_WM=128 timeout -k 10 300 python scripts/kbench.py gemm --iters 10 > gpurun_out/${TAG}_kb_wm_$i.txt 2>&1
done
