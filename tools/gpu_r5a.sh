set -o pipefail
out=gpurun_out/r5a
mkdir -p $out
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_bench_ranks.py tests/test_gpu_config4.py "tests/test_gpu_evaluate.py::test_stress_full_size_matches_oracle" "tests/test_gpu_bench_parity.py::test_stress_chain_run_follows_host" > $out/tests.log 2>&1 || { echo "gpu tests failed"; tail -60 $out/tests.log; exit 1; }
tail -15 $out/tests.log
