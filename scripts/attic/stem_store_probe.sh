# Same-box A/B of the stem conv2 epilogue: LDS-staged 16-B stores (the tree) vs the direct
# 2-byte stores (ab_c = previous HEAD, built): stem GPU tests on the tree, kbench stem
# alternating, then bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-ssp}
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_stem_fold_gpu.py -k "stem" > $R/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_c && timeout -k 10 300 python scripts/kbench.py stem --iters 10) > $R/${TAG}_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py stem --iters 10 > $R/${TAG}_tree_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_c && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > $R/${TAG}_bbase_$i.json 2> $R/${TAG}_bbase_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/${TAG}_bnew_$i.json 2> $R/${TAG}_bnew_$i.err
done
