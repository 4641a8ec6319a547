set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gelu_backward_epilogue or dropout_masks or gemm" > gpurun_out/gemm_tests.log 2>&1
A="scripts/kbench.py gemm --batch 32 --iters 1 --only s0"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gpmc_p3 -o run --output-format csv -- python $A > gpurun_out/gpmc_p3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/gpmc_p4 -o run --output-format csv -- python $A > gpurun_out/gpmc_p4.log 2>&1
bash scripts/pmc_kernel.sh gpmc scripts/kbench.py gemm --batch 32 --iters 1 --only "s0 expand"
python scripts/pmc_sum.py gpurun_out/gpmc > gpurun_out/gpmc_sum.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/gstat -o run -- python3 scripts/kbench.py gemm --batch 256 --iters 2 > gpurun_out/gemm_shapes.log 2>&1
