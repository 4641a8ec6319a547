# forward occupancy variants (SM_ATTN_FWD_WPS 2/3/4) vs the baseline worktree, per-kernel rocprof stats
set -e
TAG=${1:-r03d}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "attention" > gpurun_out/${TAG}_tests.log 2>&1
SM_ATTN_FWD_WPS=4 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "attention_dropout" > gpurun_out/${TAG}_tests4.log 2>&1
(cd ab_base && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pbase -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3) > gpurun_out/${TAG}_kb_base.log 2>&1
for w in 2 3 4; do
SM_ATTN_FWD_WPS=$w timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pnew$w -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3 > gpurun_out/${TAG}_kb_new$w.log 2>&1
done
