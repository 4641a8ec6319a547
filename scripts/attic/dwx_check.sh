set -e
TAG=${1:-r02x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or linear or layernorm or gelu or weight_grad" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -u scripts/kbench.py dwx > gpurun_out/${TAG}_dwx.txt 2>&1
timeout -k 10 200 python -u scripts/kbench.py dw > gpurun_out/${TAG}_dw.txt 2>&1
