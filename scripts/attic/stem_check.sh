set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "conv3x3 or stem" tests/test_c2_bf16_gpu.py -k "conv3x3 or stem or bf16_step or full_c2" > gpurun_out/stem_tests.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/stem_bench.json 2> gpurun_out/stem_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/stem_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/stem_prof_bench.json 2> gpurun_out/stem_prof_bench.err
