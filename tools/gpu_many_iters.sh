# many-chains leg: 1000 vs 5000 proposals per launch (256 chains)
set -e
mkdir -p gpurun_out
A="--steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-stress --no-dropin --no-config4"
for it in 1000 5000 1000 5000; do
  timeout -k 10 200 python bench.py $A --batch-iters $it >> gpurun_out/many_$it.log 2>&1
done
