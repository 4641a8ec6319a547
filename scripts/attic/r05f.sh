# round 5 / f: side-stream weight gradients (bit identity, allocator diagnostics, bounded vs
# unbounded lag) + the statistics GEMM's DPP reduction (GEMM tests, kbench bnstats)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05f}
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_wgrad_stream_gpu.py \
  tests/test_kernels_gpu.py -k "wgrad or bn_stats or persistent or gemm_layouts or linear" > gpurun_out/${T}_tests.log 2>&1 || exit 1
timeout -k 10 200 python scripts/kbench.py bnstats > gpurun_out/${T}_bnstats.log 2>&1 || exit 1
export SM_BENCH_MEMSTATS=1
for i in 1 2; do
  SM_WGRAD_STREAM=0 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_off_$i.json 2> gpurun_out/${T}_bench_off_$i.err || exit 1
  SM_WGRAD_STREAM=1 timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${T}_bench_on_$i.json 2> gpurun_out/${T}_bench_on_$i.err || exit 1
done
SM_WGRAD_STREAM=1 SM_WGRAD_LAG=0 timeout -k 10 400 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${T}_bench_unb.json 2> gpurun_out/${T}_bench_unb.err || exit 1
