# attention + dW tests, same-box A/B of attention and weight-gradient micro-benchmarks (ab_base = baseline
# worktree), bench line of the tree
set -e
TAG=${1:-r03g}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "attention or attn or dw or linear" > gpurun_out/${TAG}_tests.log 2>&1
(cd ab_base && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pbase -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3) > gpurun_out/${TAG}_kb_base.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pnew -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3 > gpurun_out/${TAG}_kb_new.log 2>&1
(cd ab_base && timeout -k 10 300 python scripts/kbench.py dw --iters 3) > gpurun_out/${TAG}_dw_base.log 2>&1
timeout -k 10 300 python scripts/kbench.py dw --iters 3 > gpurun_out/${TAG}_dw_new.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
