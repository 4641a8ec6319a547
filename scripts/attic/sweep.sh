set -e
for b in 4 16 64; do
  timeout -k 10 300 python bench.py --batch $b --steps 3 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep.log 2>&1
done
