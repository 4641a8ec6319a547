# streaming-kernel tests + one MBConv kbench A/B round (ab_base vs this tree) + the default bench line
set -e
TAG=${1:-r03y}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "dw or mbconv or MBConv or bn or se_ or batchnorm" > gpurun_out/${TAG}_tests.log 2>&1
(cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5) > gpurun_out/${TAG}_kb_base1.log 2>&1
timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_kb_new1.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
