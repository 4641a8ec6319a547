# per-kernel A/B of the attention backward's MFMA shape inside the step (rocprofv3 kernel stats)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-r06l}
for sh in 32,32 16,16 16,32 32,32 16,16; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_$sh -o run --output-format csv -- python bench.py --no-cpu-baseline --no-calibration --steps 3 --warmup 1 --attn-bwd-shape $sh > gpurun_out/${T}_prof_bench_$sh.json 2> gpurun_out/${T}_prof_bench_$sh.err
  python scripts/stepprof.py gpurun_out/${T}_prof_$sh --top 40 >> gpurun_out/${T}_summary_$sh.txt
done
