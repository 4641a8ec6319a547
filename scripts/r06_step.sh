set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06r}
timeout -k 10 600 python -u -m pytest -x -q --timeout 900 --timeout-method thread tests/test_c2_bf16_gpu.py -k "c1_batch" > gpurun_out/${T}_tests.log 2>&1
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 400 python scripts/kbench.py attn --only dec --bwd-shapes 16,18,19 --rounds 3 --iters 3 > gpurun_out/${T}_kbench_iglp.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err
python scripts/stepprof.py gpurun_out/${T}_prof --top 40 > gpurun_out/${T}_step_kernels.txt
