# one stress-chain iteration: phase cycles at 10k rays x 20k cells, then the chain tests
set -e
mkdir -p gpurun_out
timeout -k 10 300 python profiles/chain_phases.py 20000 2000 10000 > gpurun_out/ph_stress.json 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_chain.log 2>&1
