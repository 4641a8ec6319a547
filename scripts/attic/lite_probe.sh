set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_model_gpu.py -k "fp32_step" > gpurun_out/lite_tests.log 2>&1
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --lite 0 > gpurun_out/lite0.json 2> gpurun_out/lite0.err || echo "lite0 failed"
timeout -k 10 300 python bench.py --steps 4 --warmup 2 --no-cpu-baseline --lite none > gpurun_out/lite_none.json 2> gpurun_out/lite_none.err
