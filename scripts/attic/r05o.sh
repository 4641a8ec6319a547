# round 5 / o: attention forward row sums as packed pairs -- attention tests, then the library A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/r05o_tests.log 2>&1 || exit 1
bash scripts/ab_lib.sh r05o attn
