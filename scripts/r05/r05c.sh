# round 5 / c: persistent short-sequence attention backward -- bit-identity tests, kernel A/B, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05c}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "persistent or attention" > gpurun_out/${T}_tests.log 2>&1 || exit 1
for i in 1 2; do
  for v in 0 1; do
    SM_ATTN_PERS=$v timeout -k 10 200 python scripts/kbench.py attn --only enc > gpurun_out/${T}_attn_${v}_$i.log 2>&1 || exit 1
  done
done
for i in 1 2; do
  for v in 0 1; do
    SM_ATTN_PERS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_${v}_$i.json 2> gpurun_out/${T}_bench_${v}_$i.err || exit 1
  done
done
