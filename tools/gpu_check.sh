set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_exact_sum.py -x -q > gpurun_out/t_sum.log 2>&1 || { echo "sum tests failed"; exit 1; }
timeout -k 10 600 python -m pytest tests/test_gpu_chain.py -x -q > gpurun_out/t_chain.log 2>&1 || { echo "chain tests failed"; exit 1; }
timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > gpurun_out/phases5000.json 2>&1 || { echo "phases failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --batch-chains 0 --no-stress --no-full-evaluate > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
