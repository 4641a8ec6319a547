# golden parity with resident stages + bench peak memory / time per resident policy
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread -k "golden" > gpurun_out/res_tests.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --resident 1,2 > gpurun_out/res_12.json 2>&1
