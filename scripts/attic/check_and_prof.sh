# usage: bash scripts/check_and_prof.sh TAG BATCH
set -e
TAG=${1:-p}
B=${2:-64}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -q -m gpu -x > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG} -o run --output-format csv -- python bench.py --batch $B --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
