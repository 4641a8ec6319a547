# same-box full-step A/B (ab_base vs this tree, alternated twice), then the GEMM tile-variant probe
set -e
TAG=${1:-r03g2}
bash scripts/ab_bench.sh ${TAG}ab
bash scripts/r03_gemm_var.sh ${TAG}
