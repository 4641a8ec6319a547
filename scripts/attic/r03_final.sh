# round-end measurement set at this tree: full GPU test suite, then scripts/measure.sh
# (bench line, rocprof kernel stats, ledger, PMC FETCH/WRITE traffic)
set -e
TAG=${1:-r03f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
bash scripts/measure.sh ${TAG}
