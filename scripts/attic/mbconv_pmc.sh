# Stage-0 MBConv streaming kernels: TB/s at the bench shape, then HBM bytes
# (FETCH_SIZE / WRITE_SIZE, separate passes) and SQ/LDS counters at batch 32.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python scripts/kbench.py mbconv --batch 256 --iters 3 > gpurun_out/mbconv_kbench.txt 2>&1
A="scripts/kbench.py mbconv --batch 32 --iters 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/mbpmc_p3 -o run --output-format csv -- python $A > gpurun_out/mbpmc_p3.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/mbpmc_p4 -o run --output-format csv -- python $A > gpurun_out/mbpmc_p4.log 2>&1
bash scripts/pmc_kernel.sh mbpmc $A
python scripts/pmc_sum.py gpurun_out/mbpmc > gpurun_out/mbpmc_sum.txt
