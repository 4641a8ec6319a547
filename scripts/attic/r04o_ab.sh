# Same-box A/B: depthwise forward / backward kernels at 3 waves per SIMD (launch bounds
# (256, 3): 168 VGPRs with a little scratch) against ab_base (2 waves per SIMD).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04o}
true
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5) > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
