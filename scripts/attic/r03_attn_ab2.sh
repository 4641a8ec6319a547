# A/B of the decoder attention kernels: baseline worktree vs this tree (fwd / dQ at 2 and 3 waves per SIMD),
# per-kernel times from rocprofv3 --kernel-trace --stats
set -e
TAG=${1:-r03c}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "attention" > gpurun_out/${TAG}_tests.log 2>&1
(cd ab_base && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_pbase -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3 --only dec) > gpurun_out/${TAG}_kb_base.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pnew2 -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3 --only dec > gpurun_out/${TAG}_kb_new2.log 2>&1
SM_ATTN_FWD_WPS=3 SM_ATTN_DQ_WPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pnew3 -o run --output-format csv -- python scripts/kbench.py attn --drop 0.1 --iters 3 --only dec > gpurun_out/${TAG}_kb_new3.log 2>&1
for d in pbase pnew2 pnew3; do python scripts/profsum.py gpurun_out/${TAG}_$d/* 8 > gpurun_out/${TAG}_$d.txt 2>&1 || true; done
