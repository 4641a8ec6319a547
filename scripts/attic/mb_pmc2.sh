set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash scripts/pmc_kernel.sh dwbpmc scripts/kbench.py mbconv --batch 32 --iters 1
python scripts/pmc_sum.py gpurun_out/dwbpmc > gpurun_out/dwbpmc_sum.txt
