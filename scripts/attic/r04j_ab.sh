# Same-box A/B of the 16-B attention epilogue stores (ab_base = previous HEAD): attention GPU
# tests on the tree, kbench attn (all three shapes) alternating, then bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04j}
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention or attn" > $R/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py attn --iters 5) > $R/${TAG}_a_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py attn --iters 5 > $R/${TAG}_a_new_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > $R/${TAG}_base_$i.json 2> $R/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/${TAG}_new_$i.json 2> $R/${TAG}_new_$i.err
done
