set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python bench.py --batch 64 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof1.log 2>&1
