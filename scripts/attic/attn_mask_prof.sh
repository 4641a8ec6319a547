# Per-kernel times (rocprofv3 kernel trace) and SQ counters of the decoder attention
# backward, ab_base (previous HEAD) vs the tree.   usage: bash scripts/attn_mask_prof.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
TAG=${1:-mpf}
R=$GRAFT_REPO_ROOT/gpurun_out
(cd ab_base && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/${TAG}_kt_base -o run --output-format csv -- python scripts/kbench.py attn --only dec --iters 3) > $R/${TAG}_kt_base.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/${TAG}_kt_new -o run --output-format csv -- python scripts/kbench.py attn --only dec --iters 3 > $R/${TAG}_kt_new.log 2>&1
for v in base new; do
  if [ $v = base ]; then D=ab_base; else D=.; fi
  (cd $D && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_WAIT_ANY -d $R/${TAG}_${v}_p1 -o run --output-format csv -- python scripts/kbench.py attn --only dec --iters 1) > $R/${TAG}_${v}_p1.log 2>&1
  (cd $D && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_WAVES -d $R/${TAG}_${v}_p2 -o run --output-format csv -- python scripts/kbench.py attn --only dec --iters 1) > $R/${TAG}_${v}_p2.log 2>&1
done
