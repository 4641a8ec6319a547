# A/B of an env switch on the MBConv streaming-op micro-bench: bash scripts/mb_ab.sh TAG VAR "v0 v1"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=$1; VAR=$2; VALS=${3:-"0 1"}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q -x -k "dwconv or se_ or bn" --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || exit 1
for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python scripts/kbench.py mbconv --iters 5 > gpurun_out/${TAG}_${v}.log 2>&1 || exit 1
done
