# session start: GPU tests at HEAD, the default bench line, and the GEMM write-rate probe
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/r03t_gputests.log 2>&1
timeout -k 10 400 python bench.py > gpurun_out/r03t_bench.json 2> gpurun_out/r03t_bench.err
timeout -k 10 200 python scripts/kbench.py gemmw --iters 10 > gpurun_out/r03t_gemmw.txt 2>&1
