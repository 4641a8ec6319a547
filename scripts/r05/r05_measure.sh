# Round-5 HEAD measurement: GPU suite, smoke, bench line (with the CPU baseline), rocprofv3
# kernel stats of the bench, per-op ledger, FETCH/WRITE PMC passes (separate runs) -> traffic
# JSONs, C3 / C4 bench lines.   usage: bash scripts/r05/r05_measure.sh TAG
TAG=${1:-r05z}
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# test failures (rc 1) are reported but do not stop the measurements; anything else does
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/${TAG}_gputests.log 2>&1
rc=$?; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
set -e
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof_bench.err
timeout -k 10 300 python scripts/ledger.py --top 90 > gpurun_out/${TAG}_ledger.txt 2> gpurun_out/${TAG}_ledger.err
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/${TAG}_pmc_fetch -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/${TAG}_pmc_write -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 1 --warmup 1 > gpurun_out/${TAG}_pmc_write.log 2>&1
python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "attn_bwd_dq_bf16<64, true, 4>+attn_bwd_dkdv_bf16<64, true, 4>" gpurun_out/${TAG}_traffic.json
python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "attn_fwd_bf16<64, true>" gpurun_out/${TAG}_traffic_fwd.json
python scripts/pmc_traffic.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write "stem_conv1_band_kernel+stem_conv2_kernel" gpurun_out/${TAG}_traffic_stem.json
python scripts/pmc_table.py gpurun_out/${TAG}_pmc_fetch gpurun_out/${TAG}_pmc_write 90 > gpurun_out/${TAG}_traffic_table.txt
timeout -k 10 400 python bench.py --model small --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err
timeout -k 10 300 python bench.py --workload finetune --steps 5 --warmup 2 > gpurun_out/${TAG}_c4_bench.json 2> gpurun_out/${TAG}_c4_bench.err
