set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_dropout_unbiased_gpu.py tests/test_attn16_gpu.py > gpurun_out/r06b_tests.log 2>&1
timeout -k 10 300 python scripts/kbench.py attn --bwd-shapes 32,16 --rounds 3 --iters 3 > gpurun_out/r06b_kbench_attn.txt 2>&1
