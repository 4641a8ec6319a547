# round 5 / g: packed statistics epilogue (tests, kbench bnstats) + a kernel trace of one step
# with weight gradients on the side stream (do the two streams' kernels overlap?)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05g}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_stem_fold_gpu.py -k "bn_stats or persistent or gemm_layouts or linear or bnin or model_step" > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 200 python scripts/kbench.py bnstats > gpurun_out/${T}_bnstats.log 2>&1 || exit 1
SM_WGRAD_STREAM=1 timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/${T}_trace -o trace --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${T}_trace.log 2>&1 || exit 1
