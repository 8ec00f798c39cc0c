# same-box A/B of the drop-in leg (tools/dropin_only.py): BASE lib (default ab/libtdstar_base.so) vs the working tree,
# then the drop-in parity tests.  usage: bash tools/gpu_dropin_ab.sh OUT [base.so]
set -o pipefail
out=gpurun_out/${1:-dab}; mkdir -p $out
BASE=${2:-ab/libtdstar_base.so}
for k in 1 2; do
  for v in base head; do
    if [ $v = base ]; then export TD_LIB_PATH=$PWD/$BASE; else unset TD_LIB_PATH; fi
    timeout -k 10 120 python tools/dropin_only.py > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v$k.json').read().strip().splitlines()[-1]); i=d['incremental']; print('$v', i['us_per_proposal'], json.dumps(i['breakdown_us_per_proposal']))"
  done
done
unset TD_LIB_PATH
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py "tests/test_gpu_bench_parity.py::test_dropin_leg_follows_host" tests/test_gpu_main.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
