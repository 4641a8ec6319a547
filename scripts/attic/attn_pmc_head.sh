# SQ counters (two passes) of the attention kernels at B=32 (kbench attn), HEAD
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/pmc_kernel.sh apmc scripts/kbench.py attn --batch 32 --iters 1 && python scripts/pmc_sum.py gpurun_out/apmc > gpurun_out/apmc_sum.txt
