# Weight-gradient GEMMs (split-K over tokens): time and PMC FETCH_SIZE per split-round count.
# usage: bash scripts/dw_rounds_ab.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-dwr}
for r in 2 4 8 16; do
  SM_GEMM_SPLIT_ROUNDS=$r timeout -k 10 200 python scripts/kbench.py dw --iters 5 > gpurun_out/${TAG}_t_r$r.txt 2>&1
done
for r in 2 8; do
  SM_GEMM_SPLIT_ROUNDS=$r timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${TAG}_f_r$r -o run --output-format csv -- python scripts/kbench.py dw --iters 1 > gpurun_out/${TAG}_f_r$r.log 2>&1
done
