# Round-4 HEAD measurement: bench line, rocprofv3 kernel stats of the same command, per-op
# ledger, FETCH/WRITE PMC passes (separate runs) -> per-kernel traffic table and the
# roofline-kernel / stem traffic JSONs.   usage: bash scripts/r04_traffic.sh TAG
set -e
TAG=${1:-r04f}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err
timeout -k 10 300 python scripts/ledger.py --top 90 > gpurun_out/${TAG}_ledger.txt 2> gpurun_out/${TAG}_ledger.err
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_write.log 2>&1
python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "attn_bwd_dq_bf16<64, true, 4>+attn_bwd_dkdv_bf16<64, true, 4>" gpurun_out/${TAG}_traffic.json
python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "attn_fwd_bf16<64, true>" gpurun_out/${TAG}_traffic_fwd.json
python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "stem_conv1_band_kernel+stem_conv2_kernel" gpurun_out/${TAG}_traffic_stem.json
python scripts/pmc_table.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write 90 > gpurun_out/${TAG}_traffic_table.txt
