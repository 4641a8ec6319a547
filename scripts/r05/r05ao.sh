# round 5 / ao: BatchNorm-input A operand (IMP 11 / 12: the stage-0 block-0 expand under the folded stem BN2) in the persistent GEMM form, base = HEAD:
# GPU suite on the tree, then same-box per-kernel A/B (rocprofv3 kernel stats of the bench step),
# ab_lib/libsslmae_base.so (HEAD before the change, via SM_LIB_PATH) vs the tree, alternated twice
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05ao_tests.log 2>&1 || { tail -30 gpurun_out/r05ao_tests.log; exit 1; }
tail -2 gpurun_out/r05ao_tests.log
P="rocprofv3 --kernel-trace --stats -o run --output-format csv"
for i in 1 2; do
  (export SM_LIB_PATH=$GRAFT_REPO_ROOT/ab_lib/libsslmae_base.so; timeout -k 10 400 $P -d gpurun_out/r05ao_base$i -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05ao_base$i.json 2> gpurun_out/r05ao_base$i.err) || exit 1
  timeout -k 10 400 $P -d gpurun_out/r05ao_new$i -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r05ao_new$i.json 2> gpurun_out/r05ao_new$i.err || exit 1
done
for i in 1 2; do python scripts/abcmp.py gpurun_out/r05ao_base$i gpurun_out/r05ao_new$i 4 30; done
