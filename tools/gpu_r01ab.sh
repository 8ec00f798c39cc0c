# A/B: the round-1 snapshot vs HEAD, single chain config 3, same box.  Needs the snapshot
# built in-tree first: git worktree add -f variants/r01 93c8312 && make -C variants/r01/mcmc-in-tonga_amd/csrc
# (variants/ is git-ignored, not gpurun-ignored: it travels to the box)
set -e
mkdir -p gpurun_out
A="--steps 10 --warmup 2 --no-cpu-baseline --no-full-evaluate --no-stress --batch-chains 0"
for i in 1 2; do
  (cd variants/r01 && timeout -k 10 120 python bench.py $A) > gpurun_out/ab_r01_$i.log 2>&1
  timeout -k 10 120 python bench.py $A --no-dropin --no-config4 > gpurun_out/ab_head_$i.log 2>&1
done
