# round 5 / u: device-memory arena (csrc/arena.cpp) — GPU test, then B=256 bench arena (stage 0 resident) vs caching allocator, same box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_arena_gpu.py > gpurun_out/r05u_test.log 2>&1 || { tail -40 gpurun_out/r05u_test.log; exit 1; }
tail -3 gpurun_out/r05u_test.log
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2"
SM_BENCH_MEMSTATS=1 $B > gpurun_out/r05u_arena_1.json 2> gpurun_out/r05u_arena_1.err || { tail -30 gpurun_out/r05u_arena_1.err; exit 1; }
cat gpurun_out/r05u_arena_1.json; grep arena gpurun_out/r05u_arena_1.err
SM_BENCH_MEMSTATS=1 $B --arena off > gpurun_out/r05u_caching_1.json 2> gpurun_out/r05u_caching_1.err || exit 1
SM_BENCH_MEMSTATS=1 $B > gpurun_out/r05u_arena_2.json 2> gpurun_out/r05u_arena_2.err || exit 1
SM_BENCH_MEMSTATS=1 $B --arena off > gpurun_out/r05u_caching_2.json 2> gpurun_out/r05u_caching_2.err || exit 1
for f in gpurun_out/r05u_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['peak_mem_gib'],d['config']['resident_stages'],d['config']['lite_stages'],d.get('allocator'))"; done
