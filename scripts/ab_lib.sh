# Same-box A/B of two builds of the library: ab_lib/libsslmae_base.so (SM_LIB_PATH, the base
# arm) against the tree's build, alternating: attention / GEMM micro-benchmarks and the bench
# step.  usage: bash scripts/ab_lib.sh TAG [kbench-mode ...]
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-ab}; shift
BASE="SM_LIB_PATH=$GRAFT_REPO_ROOT/ab_lib/libsslmae_base.so"
for m in "$@"; do
  env $BASE timeout -k 10 200 python scripts/kbench.py $m > gpurun_out/${TAG}_${m}_base.log 2>&1 || exit 1
  timeout -k 10 200 python scripts/kbench.py $m > gpurun_out/${TAG}_${m}_new.log 2>&1 || exit 1
done
for i in 1 2; do
  env $BASE timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_bench_base_$i.json 2> gpurun_out/${TAG}_bench_base_$i.err || exit 1
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_bench_new_$i.json 2> gpurun_out/${TAG}_bench_new_$i.err || exit 1
done
