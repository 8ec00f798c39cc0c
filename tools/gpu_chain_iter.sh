# one chain-kernel iteration: bench A/B against the round-1 snapshot, phase cycles, chain + incremental tests
set -e
mkdir -p gpurun_out
bash tools/gpu_r01ab.sh
timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > gpurun_out/ph_head.json 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_incremental.py tests/test_gpu_config4.py -x -q --timeout 150 --timeout-method thread > gpurun_out/t_chain.log 2>&1
