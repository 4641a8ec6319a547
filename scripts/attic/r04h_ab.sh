# Same-box A/B of the RowStage swizzle (ab_base = previous HEAD): GEMM / conv / stem GPU
# tests on the tree, kbench gemm alternating base/new, then bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04h}
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_stem_fold_gpu.py -k "gemm or linear or conv or stem or bn" > $R/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py gemm --iters 5) > $R/${TAG}_g_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py gemm --iters 5 > $R/${TAG}_g_new_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > $R/${TAG}_base_$i.json 2> $R/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/${TAG}_new_$i.json 2> $R/${TAG}_new_$i.err
done
