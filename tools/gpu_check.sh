set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests/test_gpu_chain.py -x -q > gpurun_out/t_chain.log 2>&1 || { echo "chain tests failed rc=$?"; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || { echo "bench failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --chains-per-gpu 4 --swap-every 500 --batch-chains 0 --no-cpu-baseline --no-full-evaluate > gpurun_out/bench_temper.log 2>&1 || { echo "tempered bench failed"; exit 1; }
