# round 5 / k: caching-allocator settings (max_split_size_mb) vs fragmentation, stage-0 lite vs resident
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05k}
export SM_BENCH_MEMSTATS=1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2"
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:2048 $B > gpurun_out/${T}_ms2048.json 2> gpurun_out/${T}_ms2048.err || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:2048 $B --resident 0,1,2 --lite none > gpurun_out/${T}_ms2048_res012.json 2> gpurun_out/${T}_ms2048_res012.err || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $B --resident 0,1,2 --lite none > gpurun_out/${T}_ms512_res012.json 2> gpurun_out/${T}_ms512_res012.err || exit 1
PYTORCH_HIP_ALLOC_CONF=max_split_size_mb:512 $B > gpurun_out/${T}_ms512.json 2> gpurun_out/${T}_ms512.err || exit 1
