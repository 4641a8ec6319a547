# attention tests + same-box A/B of the attention micro-benchmark (ab_base = baseline worktree) + bench
set -e
TAG=${1:-r03b}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "attention or attn" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py attn --drop 0.1 --iters 3) > gpurun_out/${TAG}_kb_base_$i.log 2>&1
  timeout -k 10 300 python scripts/kbench.py attn --drop 0.1 --iters 3 > gpurun_out/${TAG}_kb_new_$i.log 2>&1
done
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
