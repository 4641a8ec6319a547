# round 5 / ar: final HEAD sanity: GPU suite, smoke, bench line
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r05ar_gputests.log 2>&1
rc=$?; tail -2 gpurun_out/r05ar_gputests.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r05ar_smoke.log 2>&1 || exit 1
tail -1 gpurun_out/r05ar_smoke.log
timeout -k 10 400 python bench.py > gpurun_out/r05ar_bench.json 2> gpurun_out/r05ar_bench.err || exit 1
cat gpurun_out/r05ar_bench.json
