# round-end check: all GPU tests, smoke, the default bench line
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/final_tests.log 2>&1
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1
