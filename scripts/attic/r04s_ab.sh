# SE + BN backward dx pass with folded per-channel constants (82 VGPRs, 5 waves/SIMD) against
# ab_base: SE / MBConv GPU tests on the tree, kbench mbconv alternating.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04s}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py tests/test_bf16_pin_gpu.py -k "se or mbconv or MBConv or stage" > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv --iters 5) > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
