# GPU suite + smoke + bench line (with the C1 CPU baseline) + rocprofv3 kernel stats of the
# bench + C3 / C4 bench lines.  Steps chained: a failure stops the call.
TAG=${1:-r04e}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# test failures (rc 1) are reported but do not stop the measurements; anything else does
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err
timeout -k 10 400 python bench.py --model small --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err
timeout -k 10 300 python bench.py --workload finetune --steps 5 --warmup 2 > gpurun_out/${TAG}_c4_bench.json 2> gpurun_out/${TAG}_c4_bench.err
