# final HEAD: full GPU suite + smoke
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06zi}
timeout -k 10 1000 python -u -m pytest -q --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/${T}_gputests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1
