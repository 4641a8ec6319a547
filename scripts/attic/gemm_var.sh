set -e
mkdir -p gpurun_out
for V in 2 3 1; do SM_GEMM_VARIANT=$V timeout -k 10 200 python3 scripts/kbench.py gemm --batch 256 --iters 3 > gpurun_out/gemm_v$V.log 2>&1; done
