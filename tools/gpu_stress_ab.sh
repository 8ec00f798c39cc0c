# same-box A/B of the stress-geometry chain (tools/stress_phases.py) and the headline, base build
# vs the working tree; then the chain parity tests on the working tree
set -o pipefail
out=gpurun_out/sab; mkdir -p $out
for k in 1 2; do
  for v in base head; do
    if [ $v = base ]; then export TD_LIB_PATH=$PWD/ab/libtdstar_base.so; else unset TD_LIB_PATH; fi
    timeout -k 10 300 python tools/stress_phases.py > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json; d=json.load(open('$out/$v$k.json')); print('$v', round(d['us_per_prop'],2), d['cycles'])"
  done
done
unset TD_LIB_PATH
TESTS=0 bash tools/gpu_ab.sh sab/ab base=ab/libtdstar_base.so head= || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_chain.py tests/test_gpu_bench_parity.py -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
