# attention parity tests + kernel bench (decoder d=64 with/without dropout, encoder d=32)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 60 -k "dropout_statistics or dropout_exact" > gpurun_out/attn_drop.log 2>&1
rc=$?; if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" --deselect tests/test_kernels_gpu.py::test_attention_dropout_statistics > gpurun_out/attn_tests.log 2>&1 && \
timeout -k 10 300 python scripts/kbench.py attn --iters 3 > gpurun_out/attn_kbench.log 2>&1 && \
timeout -k 10 300 python scripts/kbench.py attn --iters 3 --drop 0 --only dec >> gpurun_out/attn_kbench.log 2>&1
