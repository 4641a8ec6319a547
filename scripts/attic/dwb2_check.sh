set -e
TAG=${1:-r02x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "dwconv_bn_bwd" > gpurun_out/${TAG}_tests.log 2>&1

timeout -k 10 600 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
