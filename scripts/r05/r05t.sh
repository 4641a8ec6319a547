# round 5 / t: what stage-0 residency buys when memory allows (B = 128): lite (a1, a2 recomputed) vs resident (a2 kept)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="timeout -k 10 300 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --batch 128"
for i in 1 2; do
  $B --resident 1,2 --lite 0 > gpurun_out/r05t_lite_$i.json 2> gpurun_out/r05t_lite_$i.err || exit 1
  $B --resident 0,1,2 --lite none > gpurun_out/r05t_res_$i.json 2> gpurun_out/r05t_res_$i.err || exit 1
done
