# Same-box A/B, ab_base (previous HEAD) vs the tree: (1) GPU tests of the changed kernels,
# (2) stage-0 depthwise backward with the next item's x prefetched (kbench mbconv),
# (3) decoder attention backward with the dQ -> dK/dV keep-bit handoff: per-kernel trace
# and SQ counters.   usage: bash scripts/r04g_ab.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04g}
R=$GRAFT_REPO_ROOT/gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "dwconv or mbconv or attention or attn" > $R/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5) > $R/${TAG}_mb_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > $R/${TAG}_mb_new_$i.txt 2>&1
done
bash scripts/attn_mask_prof.sh ${TAG}a
