# same-box A/B of the drop-in leg: one-point queries on the host (default) vs the device server
# (TD_HOST_QUERY=0), alternating, then the drop-in parity tests.  usage: bash tools/gpu_hostq_ab.sh OUT
set -o pipefail
out=gpurun_out/${1:-hq}; mkdir -p $out
for k in 1 2 3; do
  for v in dev host; do
    if [ $v = dev ]; then export TD_HOST_QUERY=0; else unset TD_HOST_QUERY; fi
    timeout -k 10 120 python tools/dropin_only.py > $out/$v$k.json 2>&1 || { echo "$v failed"; tail $out/$v$k.json; exit 1; }
    python -c "import json; d=json.loads(open('$out/$v$k.json').read().strip().splitlines()[-1]); i=d['incremental']; print('$v', i['us_per_proposal'], json.dumps(i['breakdown_us_per_proposal']))"
  done
done
unset TD_HOST_QUERY
timeout -k 10 600 python -u -m pytest tests/test_gpu_incremental.py "tests/test_gpu_bench_parity.py::test_dropin_leg_follows_host" tests/test_gpu_main.py tests/test_host_nn.py -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1 || { echo tests failed; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
