# round-6 measurement package (bench side): the driver's bench command, rocprof kernel
# stats of a short uncalibrated bench + step table, PMC traffic of the probe pair, and
# the C3 (ViT-Small) / C4 (linear probe) bench lines
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06s}
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-calibration --steps 3 --warmup 1 > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err
python scripts/stepprof.py gpurun_out/${T}_prof --top 40 > gpurun_out/${T}_step_kernels.txt
bash scripts/pmc_traffic.sh ${T}
timeout -k 10 400 python3 bench.py --model small --no-cpu-baseline --no-calibration --steps 10 --warmup 3 > gpurun_out/${T}_c3_bench.json 2> gpurun_out/${T}_c3_bench.err
timeout -k 10 300 python3 bench.py --workload finetune --no-cpu-baseline --no-calibration --steps 20 --warmup 5 > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err
