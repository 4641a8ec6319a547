# round 5 / e: weight gradients on a side HIP stream -- bit-identity tests, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05e}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wgrad_stream_gpu.py \
  > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in 0 1; do
    SM_WGRAD_STREAM=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_${v}_$i.json 2> gpurun_out/${T}_bench_${v}_$i.err || exit 1
  done
done
