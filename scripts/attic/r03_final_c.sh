# round-end set, part C: PMC FETCH_SIZE / WRITE_SIZE passes (separate runs) and the traffic tables
set -e
TAG=${1:-r03f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_write.log 2>&1
timeout -k 10 120 python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "attn_bwd_dq_bf16<64, true>+attn_bwd_dkdv_bf16<64, true>" gpurun_out/${TAG}_traffic.json
timeout -k 10 120 python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "attn_fwd_bf16<64, true>" gpurun_out/${TAG}_traffic_fwd.json
timeout -k 10 120 python scripts/pmc_table.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write 80 > gpurun_out/${TAG}_traffic_table.txt
