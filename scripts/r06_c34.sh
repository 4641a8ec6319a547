# C3 / C4 bench lines at the final HEAD
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06zg}
timeout -k 10 400 python3 bench.py --model small --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/${T}_c3_bench.json 2> gpurun_out/${T}_c3_bench.err
timeout -k 10 300 python3 bench.py --workload finetune --no-cpu-baseline --no-calibration --steps 20 --warmup 5 > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err
