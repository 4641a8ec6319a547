# GEMM-epilogue BatchNorm statistics: kernel tests, model-level bf16 tests, then same-box per-kernel A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-abp}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "linear_bn_stats or linear_se or batchnorm or layernorm or gelu or gemm or dwconv or mbconv or pos_blend" > gpurun_out/bnst_tests.log 2>&1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py tests/test_c2_bf16_gpu.py > gpurun_out/bnst_model.log 2>&1
bash scripts/ab_prof.sh $TAG
