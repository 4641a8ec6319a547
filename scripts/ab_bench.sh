# Same-box A/B of the full bench step: ab_base/ (a git worktree of an older commit with its
# own built library) against this tree, alternating, cpu baseline off.
# baseline tree: git worktree add -f ab_base <commit> && (cd ab_base && python -c "import __graft_entry__ as g; g.build()")
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-ab}
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > gpurun_out/${TAG}_base_$i.json 2> gpurun_out/${TAG}_base_$i.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err || exit 1
done
