# one chain-kernel iteration without the round-1 snapshot: HEAD bench x2, phase cycles, chain + incremental tests
set -e
mkdir -p gpurun_out
A="--steps 10 --warmup 2 --no-cpu-baseline --no-full-evaluate --no-stress --batch-chains 0 --no-dropin --no-config4"
for i in 1 2; do timeout -k 10 120 python bench.py $A > gpurun_out/ab_head_$i.log 2>&1; done
timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > gpurun_out/ph_head.json 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_incremental.py tests/test_gpu_config4.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_chain.log 2>&1
