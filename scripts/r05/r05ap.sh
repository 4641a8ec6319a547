# round 5 / ap: BASELINE C3 (build-defined ViT-Small MAE) under the device-memory arena with stage 0 kept: the auto
# policy (all checkpointed, 180.7 GiB) vs --lite 0 vs --resident 0 (peak and clips/s), one box.  (--resident 2 runs
# out of memory: 295 GB in use at the failing request -- the arena stops with the sizes.)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 400 python bench.py --model small --no-cpu-baseline --steps 3 --warmup 1"
$B > gpurun_out/r05ap_auto.json 2> gpurun_out/r05ap_auto.err || exit 1
$B --resident none --lite 0 > gpurun_out/r05ap_lite0.json 2> gpurun_out/r05ap_lite0.err || { tail -5 gpurun_out/r05ap_lite0.err; exit 1; }
$B --resident 0 --lite none > gpurun_out/r05ap_res0.json 2> gpurun_out/r05ap_res0.err || { tail -5 gpurun_out/r05ap_res0.err; exit 1; }
$B > gpurun_out/r05ap_auto2.json 2> gpurun_out/r05ap_auto2.err || exit 1
for f in auto lite0 res0 auto2; do python -c "import json;d=json.loads(open('gpurun_out/r05ap_$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['peak_mem_gib'], d['config']['resident_stages'], d['config']['lite_stages'])"; done
