# full GPU test suite at HEAD, then the same-box step A/B of this session's start (ab_base) vs HEAD
set -e
TAG=${1:-r03s}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
bash scripts/ab_bench.sh ${TAG}ab
