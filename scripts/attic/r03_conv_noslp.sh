# conv.hip without SLP packing: depthwise / stem tests, kbench mbconv + stem A/B (ab_base = HEAD)
set -e
TAG=${1:-r03c}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "dw or mbconv or MBConv or stem or conv or se_" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
(cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 && timeout -k 10 300 python scripts/kbench.py stem --iters 5) > gpurun_out/${TAG}_kb_base$i.log 2>&1
(timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 && timeout -k 10 300 python scripts/kbench.py stem --iters 5) > gpurun_out/${TAG}_kb_new$i.log 2>&1
done
