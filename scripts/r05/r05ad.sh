# round 5 / ad: persistent GEMM form also at N = 384 (SM_GEMM_PP_MINN=384: the decoder / stage-2
# projection forward and data gradient, K = 384), same library, rocprofv3 kernel stats of the bench
# step, alternated twice on one box
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="rocprofv3 --kernel-trace --stats -o run --output-format csv"
for i in 1 2; do
  timeout -k 10 400 $P -d gpurun_out/r05ad_base$i -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05ad_base$i.json 2> gpurun_out/r05ad_base$i.err || exit 1
  (export SM_GEMM_PP_MINN=384; timeout -k 10 400 $P -d gpurun_out/r05ad_new$i -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05ad_new$i.json 2> gpurun_out/r05ad_new$i.err) || exit 1
done
for i in 1 2; do python scripts/abcmp.py gpurun_out/r05ad_base$i gpurun_out/r05ad_new$i 4 12; done
