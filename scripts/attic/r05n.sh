# round 5 / n: GEMM tile variant (SM_GEMM_VARIANT: 0 = rule (256-row), 3 = 128-row 4-wave blocks) at the step's shapes
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05n}
for v in 0 3; do
  SM_GEMM_VARIANT=$v timeout -k 10 200 python scripts/kbench.py gemm > gpurun_out/${T}_gemm_$v.log 2>&1 || exit 1
  SM_GEMM_VARIANT=$v timeout -k 10 200 python scripts/kbench.py bnstats > gpurun_out/${T}_bnstats_$v.log 2>&1 || exit 1
done
