# round-2 v2 evidence: GPU tests, smoke, default bench, rocprofv3 passes (tools/profile.sh)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/v2_tests.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v2_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/v2_bench.log 2>&1
bash tools/profile.sh ${TAG:-r02_v3} > gpurun_out/v2_prof.log 2>&1
