# attention kernel tests + same-box kbench A/B (ab_base/ vs this tree), drop 0.1 for the decoder case
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention or attn" > gpurun_out/attn_ab_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python -u scripts/kbench.py attn --iters 3) > gpurun_out/attn_ab_base_$i.txt 2>&1
  timeout -k 10 300 python -u scripts/kbench.py attn --iters 3 > gpurun_out/attn_ab_new_$i.txt 2>&1
done
