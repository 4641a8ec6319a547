# One GPU call: attention + stem-fold parity tests, attention-backward variant profiles,
# a short bench line, the bf16 pin probe.  A step that fails its assertions (rc 1) does
# not stop the call; a timeout / abort / fault (any other rc) does.
TAG=${1:-r04c}
VARS=${2:-"0 1 2 3 4"}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc $rc: $*" >> gpurun_out/${TAG}_abort.txt; exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_stem_fold_gpu.py \
  tests/test_kernels_gpu.py tests/test_c2_bf16_gpu.py -k "attention or attn or fold or bnin or bn_apply_residual or linear_dw_bn or linear_se or linear_dw_se or linear_bn_stats or dma" > gpurun_out/${TAG}_tests.log 2>&1
for v in $VARS; do
  step env SM_ATTN_BWD_VAR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_v$v -o run \
    --output-format csv -- python scripts/kbench.py attn --only dec --iters 4 > gpurun_out/${TAG}_v$v.txt 2>&1
  python scripts/profsum.py gpurun_out/${TAG}_v$v 8 >> gpurun_out/${TAG}_v$v.txt 2>&1
done
step timeout -k 10 300 python -u scripts/gemm_dma_ab.py --reps 2 > gpurun_out/${TAG}_gemm_dma.txt 2>&1
step timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
step timeout -k 10 420 python -u scripts/bf16_pin_probe.py --batch ${PIN_B:-16} > gpurun_out/${TAG}_pin.log 2>&1
