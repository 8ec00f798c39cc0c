# A/B: the round-1 snapshot (variants/r01, git worktree of 93c8312) vs HEAD, single chain config 3, same box
set -e
mkdir -p gpurun_out
A="--steps 10 --warmup 2 --no-cpu-baseline --no-full-evaluate --no-stress --batch-chains 0"
for i in 1 2; do
  (cd variants/r01 && timeout -k 10 120 python bench.py $A) > gpurun_out/ab_r01_$i.log 2>&1
  timeout -k 10 120 python bench.py $A --no-dropin --no-config4 > gpurun_out/ab_head_$i.log 2>&1
done
