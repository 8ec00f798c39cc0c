set -o pipefail
mkdir -p gpurun_out/dr
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --batch-chains 0 --no-stress --no-config4 > gpurun_out/dr/bench.log 2>&1 || { echo bench failed; tail gpurun_out/dr/bench.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/dr/bench.log').read().strip().splitlines()[-1]); print(json.dumps(d['dropin'])); print(json.dumps(d['full_evaluate']['grid']))"
