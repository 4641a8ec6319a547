# packed-GELU check: GPU tests of the touched kernels, then same-box A/B (ab_base = previous
# commit) of the stage-0 MBConv micro-benchmarks and per-kernel rocprof stats of the step
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r03l}
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py tests/test_model_gpu.py > gpurun_out/${TAG}_tests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python scripts/kbench.py mbconv) > gpurun_out/${TAG}_kb_base_$i.txt 2>&1
  timeout -k 10 300 python scripts/kbench.py mbconv > gpurun_out/${TAG}_kb_new_$i.txt 2>&1
done
bash scripts/ab_prof.sh ${TAG}_abp
