# quick GPU iteration: exact-sum + chain tests, phase profiles, short bench
set -o pipefail
mkdir -p gpurun_out/it
timeout -k 10 300 python -u -m pytest tests/test_gpu_exact_sum.py -x -q --timeout 120 --timeout-method thread > gpurun_out/it/t_sum.log 2>&1 || { echo "sum tests failed"; tail -30 gpurun_out/it/t_sum.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_chain.py -x -q --timeout 300 --timeout-method thread > gpurun_out/it/t_chain.log 2>&1 || { echo "chain tests failed"; tail -30 gpurun_out/it/t_chain.log; exit 1; }
timeout -k 10 100 python tools/lds_plan.py > gpurun_out/it/lds.txt 2>&1 || { echo lds plan failed; exit 1; }
timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > gpurun_out/it/c3.json 2>&1 || { echo "phases failed"; exit 1; }
timeout -k 10 300 python profiles/chain_phases.py 20000 2000 10000 > gpurun_out/it/stress.json 2>&1 || { echo "stress phases failed"; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --no-cpu-baseline --batch-chains 256 --no-full-evaluate --no-stress > gpurun_out/it/bench.log 2>&1 || { echo "bench failed"; tail gpurun_out/it/bench.log; exit 1; }
tail -2 gpurun_out/it/t_sum.log; tail -2 gpurun_out/it/t_chain.log; cat gpurun_out/it/lds.txt
python - <<'PY'
import json
for f in ("c3", "stress"):
    d = json.load(open("gpurun_out/it/%s.json" % f))
    print(f, round(d["us_per_iter_wall"], 2), "us/iter", {k: v["cycles_per_iter"] for k, v in d["phases"].items()})
b = json.loads(open("gpurun_out/it/bench.log").read().strip().splitlines()[-1])
print("bench", b["value"], b["roofline"]["frac"], b.get("many_chains", {}).get("proposals_per_s"))
PY
