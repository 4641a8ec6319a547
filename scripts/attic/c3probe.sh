set -e
mkdir -p gpurun_out
for r in none 2 1,2; do
  timeout -k 10 240 python bench.py --model small --steps 2 --warmup 1 --no-cpu-baseline --resident $r > gpurun_out/small_$r.json 2> gpurun_out/small_$r.err || echo "small $r failed rc=$?"
done
timeout -k 10 300 python bench.py --workload finetune --steps 5 --warmup 2 > gpurun_out/ft.json 2> gpurun_out/ft.err
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_model_gpu.py -k small > gpurun_out/t4.log 2>&1
