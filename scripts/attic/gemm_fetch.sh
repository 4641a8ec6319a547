# FETCH_SIZE / WRITE_SIZE passes (separate runs) over kbench gemm shapes at batch 32
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="scripts/kbench.py gemm --batch 32 --iters 1"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/gf_p1 -o run --output-format csv -- python $A > gpurun_out/gf_p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/gf_p2 -o run --output-format csv -- python $A > gpurun_out/gf_p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/gf_p0 -o run --output-format csv -- python $A > gpurun_out/gf_p0.log 2>&1
