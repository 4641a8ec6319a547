# round 5 / af: what the attention-probability dropout costs the decoder attention (kbench attn --only dec,
# p = 0.1 vs 0, alternated twice on one box)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for i in 1 2; do
  for p in 0.1 0.0; do
    echo "== p=$p pass $i"; timeout -k 10 200 python scripts/kbench.py attn --only dec --drop $p --iters 5 || exit 1
  done
done > gpurun_out/r05af_attn_drop_cost.txt 2>&1
cat gpurun_out/r05af_attn_drop_cost.txt
