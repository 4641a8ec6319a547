# GPU call: fold / DMA / tube tests, GEMM variant A/B + K sweep, bench line, bf16 pin probe
TAG=${1:-r04d}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { "$@"; rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step rc $rc: $*" >> gpurun_out/${TAG}_abort.txt; exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_stem_fold_gpu.py \
  tests/test_kernels_gpu.py -k "fold or bnin or bn_apply_residual or linear_dw_bn or dma or tube or attention_fwd_bwd or attention_dropout_exact" > gpurun_out/${TAG}_tests.log 2>&1
step timeout -k 10 400 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
step timeout -k 10 300 python -u scripts/gemm_dma_ab.py --reps 2 --variants 0,1,2 > gpurun_out/${TAG}_gemm_dma.txt 2>&1
step timeout -k 10 300 python -u scripts/gemm_ksweep.py --n 384,1152 --ks 128,256,384,768,1536 > gpurun_out/${TAG}_ksweep.txt 2>&1
step timeout -k 10 420 python -u scripts/bf16_pin_probe.py --batch ${PIN_B:-16} > gpurun_out/${TAG}_pin.log 2>&1
