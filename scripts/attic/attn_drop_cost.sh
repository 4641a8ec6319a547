cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/kbench.py attn --only dec --drop 0.1 --iters 3 > gpurun_out/attn_drop1.txt 2>&1 || exit 1
timeout -k 10 300 python -u scripts/kbench.py attn --only dec --drop 0.0 --iters 3 > gpurun_out/attn_drop0.txt 2>&1 || exit 1
