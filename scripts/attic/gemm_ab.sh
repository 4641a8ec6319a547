# GEMM variants: parity tests + kernel bench
# (SM_GEMM_VARIANT 1 = 128x128 v1, 2 = v2 256x128, 3 = v2 128x128)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
VARS=${VARS:-"2 3"}
for v in $VARS; do
  SM_GEMM_VARIANT=$v timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm or linear" > gpurun_out/gab_tests_$v.log 2>&1 || exit 1
done
for v in $VARS; do
  SM_GEMM_VARIANT=$v timeout -k 10 300 python scripts/kbench.py gemm --iters 5 > gpurun_out/gab_bench_$v.log 2>&1 || exit 1
done
