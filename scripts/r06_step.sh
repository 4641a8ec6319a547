set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06t}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_mf16_gpu.py tests/test_kernels_gpu.py -k "gemm or linear or mf16" > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 600 python scripts/kbench.py gemm --mf 32,16 --rounds 3 --iters 3 > gpurun_out/${T}_kbench_mf.txt 2>&1
