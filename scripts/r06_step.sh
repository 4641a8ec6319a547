set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06g}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "stem_conv2_direct" > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 300 python scripts/kbench.py stem --rounds 3 --iters 5 > gpurun_out/${T}_kbench_stem.txt 2>&1
