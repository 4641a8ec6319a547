set -e
mkdir -p gpurun_out
timeout -k 10 200 python3 scripts/kbench.py gemmk --batch 256 --iters 3 > gpurun_out/gemmk.log 2>&1
