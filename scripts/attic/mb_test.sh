set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_c2_bf16_gpu.py tests/test_model_gpu.py > gpurun_out/mb_tests.log 2>&1
timeout -k 10 300 python scripts/kbench.py mbconv --batch 256 --iters 3 > gpurun_out/mbconv_kbench.txt 2>&1
timeout -k 10 400 python bench.py > gpurun_out/bench_mb.json 2> gpurun_out/bench_mb.err
