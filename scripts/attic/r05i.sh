# round 5 / i: allocator expandable segments and the stage-0 memory policy (lite vs resident)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05i}
export SM_BENCH_MEMSTATS=1
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2"
$B > gpurun_out/${T}_base.json 2> gpurun_out/${T}_base.err || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $B > gpurun_out/${T}_exp.json 2> gpurun_out/${T}_exp.err || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $B --resident 0,1,2 --lite none > gpurun_out/${T}_exp_res012.json 2> gpurun_out/${T}_exp_res012.err || exit 1
