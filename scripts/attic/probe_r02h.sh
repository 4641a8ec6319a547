set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/kbench.py attn --drop 0.1 > gpurun_out/r02h_attn_p01.txt 2>&1
timeout -k 10 200 python -u scripts/kbench.py attn --drop 0.0 --only dec > gpurun_out/r02h_attn_p0.txt 2>&1
timeout -k 10 200 python -u scripts/kbench.py mbconv > gpurun_out/r02h_mbconv.txt 2>&1
