# phase cycles of the round-1 snapshot (variants/r01) vs HEAD, config 3
set -e
mkdir -p gpurun_out
(cd variants/r01 && timeout -k 10 200 python profiles/chain_phases.py 5000 20000) > gpurun_out/ph_r01.json 2>&1
timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > gpurun_out/ph_head.json 2>&1
