set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06zc}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_gemm_mf16_gpu.py -k "persistent or linear or gemm or mf16" > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 500 python scripts/pp_minn_ab.py --dx --rounds 5 --iters 3 > gpurun_out/${T}_pp_dx.txt 2>&1
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
