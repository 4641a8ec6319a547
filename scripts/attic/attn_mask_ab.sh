# Same-box A/B of the dQ -> dK/dV dropout keep-bit handoff (ab_base = previous HEAD, built):
# attention GPU tests on the tree, kbench dec alternating base/new, then bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-mab}
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention or attn" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 200 python scripts/kbench.py attn --only dec --iters 5) > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 200 python scripts/kbench.py attn --only dec --iters 5 > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > gpurun_out/${TAG}_base_$i.json 2> gpurun_out/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err
done
