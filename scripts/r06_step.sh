# same-box A/B: base library (ab_lib/libsslmae_base.so) vs the tree's, kernel stats of the bench step
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06n}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "dwconv" tests/test_attn16_gpu.py > gpurun_out/${T}_tests.log 2>&1
for i in 1 2; do
  SM_LIB_PATH=$GRAFT_REPO_ROOT/ab_lib/libsslmae_base.so timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_base_$i -o run --output-format csv -- python bench.py --no-cpu-baseline --no-calibration --steps 3 --warmup 1 > gpurun_out/${T}_base_$i.json 2> gpurun_out/${T}_base_$i.err
  python scripts/stepprof.py gpurun_out/${T}_base_$i --top 60 > gpurun_out/${T}_base_${i}_summary.txt
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_new_$i -o run --output-format csv -- python bench.py --no-cpu-baseline --no-calibration --steps 3 --warmup 1 > gpurun_out/${T}_new_$i.json 2> gpurun_out/${T}_new_$i.err
  python scripts/stepprof.py gpurun_out/${T}_new_$i --top 60 > gpurun_out/${T}_new_${i}_summary.txt
done
timeout -k 10 300 python scripts/kbench.py attn --only dec --fwd-shapes 32,16 --rounds 3 --iters 3 > gpurun_out/${T}_kbench_fwd.txt 2>&1
