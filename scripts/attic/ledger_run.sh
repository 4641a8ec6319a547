# per-op roofline ledger of one B=256 bench step (HIP events per kernels.* call)
set -e
TAG=${1:-r02x}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/ledger.py --top 90 > gpurun_out/${TAG}_ledger.txt 2> gpurun_out/${TAG}_ledger.err
