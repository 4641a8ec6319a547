# attention tests + per-kernel rocprof stats of the attention micro-benchmark, baseline worktree vs tree (x2)
set -e
TAG=${1:-r03f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "attention or attn" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
(cd ab_base && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pbase$i -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3) > gpurun_out/${TAG}_kb_base$i.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pnew$i -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3 > gpurun_out/${TAG}_kb_new$i.log 2>&1
done
