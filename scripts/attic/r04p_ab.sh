# Depthwise forward with the extended ring (next band's rows committed into slots of
# their own during the current band: one barrier per band) against the two-barrier ring
# (SM_DWF_XR=0), same build, alternating; MBConv / depthwise GPU tests on the default.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04p}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "dw or depthwise or mbconv or MBConv" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  SM_DWF_XR=0 timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
