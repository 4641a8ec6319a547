# stem BN2 fold tests + bf16-vs-fp32 pin probe + a short bench line
set -e
TAG=${1:-r04c}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_stem_fold_gpu.py > gpurun_out/${TAG}_fold_tests.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 900 python -u scripts/bf16_pin_probe.py --batch ${PIN_B:-32} > gpurun_out/${TAG}_pin.log 2>&1
