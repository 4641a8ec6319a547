cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/kbench.py dwse --iters 5 > gpurun_out/dwse_bench.txt 2>&1
