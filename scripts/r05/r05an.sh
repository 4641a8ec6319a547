# round 5 / an: VERDICT r4 item 4's GELU A/B -- the forward GELU as an odd-polynomial erf (10 Horner terms on z^2,
# z clamped to +-3: 2e-5 absolute on Phi) against the A&S 7.1.26 rcp + exp2 form, same box: kbench mbconv (the
# stage-0 streaming ops; the derivative sites keep the exp form), base = HEAD (SM_LIB_PATH) vs the polynomial
# build, alternated twice.  Timing only: the polynomial build is not kept (forward and recompute sites would differ).
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
BASE="SM_LIB_PATH=$GRAFT_REPO_ROOT/ab_lib/libsslmae_base.so"
for i in 1 2; do
  echo "== base $i"; env $BASE timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 || exit 1
  echo "== poly $i"; timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 || exit 1
done > gpurun_out/r05an_gelu_poly_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/r05an_gelu_poly_ab.txt
