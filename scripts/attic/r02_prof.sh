# bench line + rocprofv3 kernel stats of the same command + per-step summary + per-op ledger
set -e
TAG=${1:-r02x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err
python scripts/stepprof.py gpurun_out/${TAG}_prof --top 45 > gpurun_out/${TAG}_summary.txt
timeout -k 10 300 python -u scripts/ledger.py --top 90 > gpurun_out/${TAG}_ledger.txt 2> gpurun_out/${TAG}_ledger.err
