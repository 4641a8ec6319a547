# Same-box per-kernel A/B: rocprofv3 kernel stats of the bench step for ab_base/ and this tree
set -e
# baseline tree: git worktree add -f ab_base <commit> && (cd ab_base && python -c "import __graft_entry__ as g; g.build()")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-abp}
(cd ab_base && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_base -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_base.json 2> $GRAFT_REPO_ROOT/gpurun_out/${TAG}_base.err)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_new -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_new.json 2> gpurun_out/${TAG}_new.err
