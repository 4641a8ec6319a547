# round 5 / s: caching-allocator segments after a bench run (fragmentation diagnosis)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SM_BENCH_MEMSTATS=1 SM_BENCH_SNAPSHOT=gpurun_out/r05s_snapshot.json timeout -k 10 300 python bench.py --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/r05s_bench.json 2> gpurun_out/r05s_bench.err || exit 1
