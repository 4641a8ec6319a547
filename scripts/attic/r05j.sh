# round 5 / j: which allocator setting does this PyTorch-ROCm build honour (expandable segments)?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r05j}
P="timeout -k 10 120 python scripts/r05/alloc_probe.py"
$P env > gpurun_out/${T}.log 2>&1 || exit 1
PYTORCH_HIP_ALLOC_CONF=expandable_segments:True $P env >> gpurun_out/${T}.log 2>&1 || exit 1
PYTORCH_CUDA_ALLOC_CONF=expandable_segments:True $P env >> gpurun_out/${T}.log 2>&1 || exit 1
PYTORCH_ALLOC_CONF=expandable_segments:True $P env >> gpurun_out/${T}.log 2>&1 || exit 1
$P api >> gpurun_out/${T}.log 2>&1 || exit 1
