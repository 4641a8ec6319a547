# round 5 / l: double-buffered dK/dV (one barrier per tile) -- bit identity, attention tests under it, kernel + step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05l}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/${T}_tests.log 2>&1 || exit 1
SM_ATTN_DB=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "attention" > gpurun_out/${T}_tests_db.log 2>&1 || exit 1
for v in 0 1; do
  SM_ATTN_DB=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$v -o p -- python3 scripts/kbench.py attn > gpurun_out/${T}_attn_$v.log 2>&1 || exit 1
done
for i in 1 2; do
  for v in 0 1; do
    SM_ATTN_DB=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_${v}_$i.json 2> gpurun_out/${T}_bench_${v}_$i.err || exit 1
  done
done
