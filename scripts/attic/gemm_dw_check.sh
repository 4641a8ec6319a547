# GEMM parity tests + weight-gradient micro-bench + per-op ledger
set -e
TAG=${1:-r02x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or linear or conv3x3 or colsum" > gpurun_out/${TAG}_gemmtests.log 2>&1
timeout -k 10 200 python -u scripts/kbench.py dw > gpurun_out/${TAG}_dw.txt 2>&1
timeout -k 10 300 python -u scripts/ledger.py --top 90 > gpurun_out/${TAG}_ledger.txt 2> gpurun_out/${TAG}_ledger.err
