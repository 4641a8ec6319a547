# LayerNorm backward at 32 lanes per row for C = 384: full GPU suite on the tree, then
# bench steps alternating with ab_base (previous HEAD, built) and the per-kernel stats of both.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-r04r}
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
for i in 1 2; do
  (cd ab_base && timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2) > gpurun_out/${TAG}_base_$i.json 2> gpurun_out/${TAG}_base_$i.err
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_new_$i.json 2> gpurun_out/${TAG}_new_$i.err
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof_new -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
cd ab_base && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d ../gpurun_out/${TAG}_prof_base -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 > /dev/null 2>&1
