# Same-box A/B of the 8-wave encoder attention backward (d = 32, L >= 2048) against ab_base
# (previous HEAD, built): attention GPU tests on the tree, kbench enc1 alternating, bench steps.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04m}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 200 python scripts/kbench.py attn --only enc1 --iters 10) > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 200 python scripts/kbench.py attn --only enc1 --iters 10 > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > gpurun_out/${TAG}_base_$i.json 2> gpurun_out/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err
done
