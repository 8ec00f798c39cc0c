# same-box A/B of the stress-geometry chain (tools/stress_phases.py: 10k rays x 20k cells, phase stamps):
# BASE lib (default ab/libtdstar_base.so) vs the working tree, alternating; then the HBM-layout parity
# tests.  usage: bash tools/gpu_stress_ab.sh OUT [base.so]
set -o pipefail
out=gpurun_out/${1:-sab}; mkdir -p $out
BASE=${2:-ab/libtdstar_base.so}
for k in 1 2; do
  for v in base head; do
    if [ $v = base ]; then export TD_LIB_PATH=$PWD/$BASE; else unset TD_LIB_PATH; fi
    timeout -k 10 200 python tools/stress_phases.py > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json; d=json.load(open('$out/$v$k.json')); print('$v', round(d['us_per_prop'],2), d['cycles'], {a: d['by_action'][a]['D'] for a in d['by_action']}, d['diag']['15'])"
  done
done
unset TD_LIB_PATH
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py "tests/test_gpu_bench_parity.py::test_stress_chain_run_follows_host" "tests/test_gpu_bench_parity.py::test_stress_subset_chain_matches_oracle" -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
