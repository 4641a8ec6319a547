# depthwise tests + one MBConv kbench A/B round (ab_base vs this tree), then the default bench
# line and rocprofv3 kernel stats of the bench at this tree
set -e
TAG=${1:-r03x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "dw or mbconv or MBConv" > gpurun_out/${TAG}_tests.log 2>&1
(cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5) > gpurun_out/${TAG}_kb_base1.log 2>&1
timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_kb_new1.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err
