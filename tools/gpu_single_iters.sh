# single chain: 5000 vs 20000 proposals per launch (one step = one launch)
set -e
mkdir -p gpurun_out
A="--no-cpu-baseline --no-full-evaluate --no-stress --no-dropin --no-config4 --batch-chains 0"
for r in 1 2; do
  timeout -k 10 200 python bench.py $A --steps 8 --warmup 2 --iters-per-step 5000 >> gpurun_out/single_5000.log 2>&1
  timeout -k 10 200 python bench.py $A --steps 2 --warmup 1 --iters-per-step 20000 >> gpurun_out/single_20000.log 2>&1
done
