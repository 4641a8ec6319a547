# Same-box A/B of the 2-wave attention blocks at L = 784 (ab_base = previous HEAD, built):
# attention GPU tests on the tree, then kbench enc2 alternating base/new, then bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-nwab}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 200 python scripts/kbench.py attn --only enc2 --iters 10) > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 200 python scripts/kbench.py attn --only enc2 --iters 10 > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > gpurun_out/${TAG}_base_$i.json 2> gpurun_out/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err
done
