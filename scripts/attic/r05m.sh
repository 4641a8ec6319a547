# round 5 / m: 512-row GEMM blocks (16 waves, one block per CU) -- bit identity, kernel A/B, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05m}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "bm512 or persistent or gemm_layouts" > gpurun_out/${T}_tests.log 2>&1 || exit 1
for v in 0 1; do
  SM_GEMM_BM512=$v timeout -k 10 200 python scripts/kbench.py gemm > gpurun_out/${T}_gemm_$v.log 2>&1 || exit 1
  SM_GEMM_BM512=$v timeout -k 10 200 python scripts/kbench.py gemmk > gpurun_out/${T}_gemmk_$v.log 2>&1 || exit 1
done
for i in 1 2; do
  for v in 0 1; do
    SM_GEMM_BM512=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_${v}_$i.json 2> gpurun_out/${T}_bench_${v}_$i.err || exit 1
  done
done
