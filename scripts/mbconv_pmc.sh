# SQ counters (two passes) + FETCH/WRITE of the stage-0 MBConv streaming kernels at B=64
# (kbench mbconv: 512 frames of 112x112x384).   usage: bash scripts/mbconv_pmc.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-mbp}
timeout -k 10 200 python scripts/kbench.py mbconv --batch 64 --iters 5 > gpurun_out/${TAG}_kbench.txt 2>&1
bash scripts/pmc_kernel.sh ${TAG} scripts/kbench.py mbconv --batch 64 --iters 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${TAG}_fetch -o run --output-format csv -- python scripts/kbench.py mbconv --batch 64 --iters 1 > gpurun_out/${TAG}_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${TAG}_write -o run --output-format csv -- python scripts/kbench.py mbconv --batch 64 --iters 1 > gpurun_out/${TAG}_write.log 2>&1
