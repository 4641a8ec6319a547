# attention + GEMM tests, then kbench attn and gemm A/B (ab_base vs this tree), alternated twice
set -e
TAG=${1:-r03z}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -m gpu -k "attention or attn or gemm or linear" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
(cd ab_base && timeout -k 10 300 python scripts/kbench.py attn --drop 0.1 --iters 5) > gpurun_out/${TAG}_ka_base$i.log 2>&1
timeout -k 10 300 python scripts/kbench.py attn --drop 0.1 --iters 5 > gpurun_out/${TAG}_ka_new$i.log 2>&1
(cd ab_base && timeout -k 10 300 python scripts/kbench.py gemm --iters 5) > gpurun_out/${TAG}_kg_base$i.log 2>&1
timeout -k 10 300 python scripts/kbench.py gemm --iters 5 > gpurun_out/${TAG}_kg_new$i.log 2>&1
done
