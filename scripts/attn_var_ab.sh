# Same-box A/B of attention-backward variants (SM_ATTN_BWD_VAR, csrc/attention.hip
# launch_attn_bwd): attention tests per variant, then rocprofv3 kernel stats of the
# decoder attention micro-benchmark per variant, alternating twice.
# usage: bash scripts/attn_var_ab.sh TAG "0 1 2 3"
set -e
TAG=${1:-attnab}
VARS=${2:-"0 1 2 3 4"}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in $VARS; do
  SM_ATTN_BWD_VAR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention or attn" > gpurun_out/${TAG}_test_v$v.log 2>&1
done
for rep in 1 2; do
  for v in $VARS; do
    SM_ATTN_BWD_VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_v${v}_r$rep -o run \
      --output-format csv -- python scripts/kbench.py attn --only ${ONLY:-dec} --iters 4 > gpurun_out/${TAG}_v${v}_r$rep.txt 2>&1
    python scripts/profsum.py gpurun_out/${TAG}_v${v}_r$rep 8 >> gpurun_out/${TAG}_v${v}_r$rep.txt 2>&1 || true
  done
done
