set -e
TAG=${1:-r02x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_c2_bf16_gpu.py tests/test_kernels_gpu.py -k "mbconv_fused_middle or dwconv" > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -u scripts/kbench.py mbconv > gpurun_out/${TAG}_mbconv.txt 2>&1
