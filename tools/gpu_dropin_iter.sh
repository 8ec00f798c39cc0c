# drop-in incremental path: tests and the bench's dropin leg
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_incremental.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_inc.log 2>&1
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-stress --batch-chains 0 --no-config4 > gpurun_out/dropin_$i.log 2>&1
done
