# stress phases + config-3 A/B + chain/incremental tests
set -e
mkdir -p gpurun_out
timeout -k 10 300 python profiles/chain_phases.py 20000 2000 10000 > gpurun_out/ph_stress.json 2>&1
bash tools/gpu_chain_iter.sh
