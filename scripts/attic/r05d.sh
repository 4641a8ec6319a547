# round 5 / d: stem conv2 from the clip (a1 not in HBM) -- bit-identity tests, kernel times, step A/B
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05d}
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "stem" > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 200 python scripts/kbench.py stem --batch 256 > gpurun_out/${T}_stem.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_stem_fold_gpu.py \
  tests/test_bf16_pin_gpu.py > gpurun_out/${T}_pin.log 2>&1 || exit 1
for i in 1 2; do
  for v in 0 1; do
    SM_STEM_FROM_CLIP=$v timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_${v}_$i.json 2> gpurun_out/${T}_bench_${v}_$i.err || exit 1
  done
done
