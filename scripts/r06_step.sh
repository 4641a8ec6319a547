set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06zm}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_dw384_gpu.py > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 400 python scripts/dw384_ab.py --key dw384_notr --rounds 5 --iters 3 > gpurun_out/${T}_dw384.txt 2>&1
