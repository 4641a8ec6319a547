set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_finetune_gpu.py tests/test_driver_gpu.py tests/test_driver_dp_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "small or ft_ssl or droppath or rng or main or linear_probe" > gpurun_out/r03a_tests.log 2>&1
timeout -k 10 300 python scripts/blas_cmp.py > gpurun_out/r03a_blas.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err
