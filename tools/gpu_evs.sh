# The resident full evaluate on the GPU: its tests, then its timing against the launches.
#   bash tools/gpu_evs.sh OUT
set -o pipefail
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eval_server.py -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "eval-server tests rc=$rc: $(tail -1 $out/tests.log)"
if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit 1; fi
timeout -k 10 120 python -u tools/eval_server_time.py 400 > $out/time.json 2> $out/time.err
rc2=$?
echo "timing rc=$rc2"; cat $out/time.json
exit $rc
