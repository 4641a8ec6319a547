# attention parity at small and bench shapes + decoder/encoder kernel timings
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention or attn" > gpurun_out/attn_tests.log 2>&1
timeout -k 10 200 python3 scripts/kbench.py attn --batch 256 --drop 0.1 --iters 3 > gpurun_out/attn_kb.log 2>&1
