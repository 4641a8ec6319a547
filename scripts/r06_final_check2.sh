# round-6 closing check at HEAD: GPU suite, smoke, the driver's bench command, kernel stats
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06x}
timeout -k 10 1000 python -u -m pytest -q --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/${T}_gputests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
timeout -k 10 500 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-calibration --steps 3 --warmup 1 > gpurun_out/${T}_prof_bench.json 2> gpurun_out/${T}_prof_bench.err
python scripts/stepprof.py gpurun_out/${T}_prof --top 40 > gpurun_out/${T}_step_kernels.txt
