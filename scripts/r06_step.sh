set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06zh}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "persistent or linear_dx or gelu" > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 400 python scripts/kbench.py dxgelu --rounds 5 --iters 3 > gpurun_out/${T}_kbench_dxgelu.txt 2>&1
