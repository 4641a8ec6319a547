# SE-operand projection GEMMs (forward A operand, weight-gradient B operand): kernel tests + micro-bench
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "linear or gemm or se_ or layernorm" > gpurun_out/dwse_tests.log 2>&1
timeout -k 10 200 python -u scripts/kbench.py dwse --iters 5 > gpurun_out/dwse_bench.txt 2>&1
