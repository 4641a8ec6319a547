# BASELINE C3 (ViT-Small MAE, 256 clips on one GPU) and C4 (frozen-encoder fine-tune) bench lines
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-c3c4}
timeout -k 10 500 python bench.py --model small --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/${TAG}_small.json 2> gpurun_out/${TAG}_small.err
timeout -k 10 400 python bench.py --workload finetune --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/${TAG}_finetune.json 2> gpurun_out/${TAG}_finetune.err
