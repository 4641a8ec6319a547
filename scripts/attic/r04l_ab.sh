# Same-box A/B of the next-pixel prefetch in the SE (+BN) streaming kernels (ab_c = earlier
# HEAD, built): SE / MBConv GPU tests on the tree, kbench mbconv alternating, bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04l}
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "se or mbconv or dwconv" > $R/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_c && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5) > $R/${TAG}_m_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > $R/${TAG}_m_new_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_c && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > $R/${TAG}_base_$i.json 2> $R/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > $R/${TAG}_new_$i.json 2> $R/${TAG}_new_$i.err
done
