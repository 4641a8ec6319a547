# round 5 / aj: tiles per block of the persistent GEMM form, step-level A/B on one box (rocprofv3 kernel stats of the
# bench step): K <= 128 at 8 (default) vs 16 tiles, K <= 384 at 2 (default) vs 3 tiles
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
P="rocprofv3 --kernel-trace --stats -o run --output-format csv"
arm() { (export $2; timeout -k 10 400 $P -d gpurun_out/r05aj_$1 -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05aj_$1.json 2> gpurun_out/r05aj_$1.err); }
for i in 1 2; do
  arm base$i "SM_NONE=1" || exit 1
  arm s16_$i "SM_GEMM_PP_ROUNDS_SMALLK=16" || exit 1
  arm m3_$i "SM_GEMM_PP_ROUNDS_MIDK=3" || exit 1
done
for i in 1 2; do python scripts/abcmp.py gpurun_out/r05aj_base$i gpurun_out/r05aj_s16_$i 4 6; python scripts/abcmp.py gpurun_out/r05aj_base$i gpurun_out/r05aj_m3_$i 4 6; done
