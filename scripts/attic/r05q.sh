# round 5 / q: 8-wave staggered dK/dV (waves 4-7 one query half behind) -- bit identity, attention tests under it, kernel + step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05q}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/${T}_tests.log 2>&1 || exit 1
SM_ATTN_STAG=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/${T}_tests_stag.log 2>&1 || exit 1
for v in 0 1; do
  SM_ATTN_STAG=$v timeout -k 10 200 python scripts/kbench.py attn --only dec > gpurun_out/${T}_attn_$v.log 2>&1 || exit 1
done
for i in 1 2; do
  for v in 0 1; do
    SM_ATTN_STAG=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_${v}_$i.json 2> gpurun_out/${T}_bench_${v}_$i.err || exit 1
  done
done
