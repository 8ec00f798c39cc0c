# td_evaluate's full path: its parity tests on the in-tree build (NOTESTS=1 skips them), then
# tools/eval_time.py per library variant:  bash tools/gpu_eval_ab.sh OUT name=lib.so ... ("-": in-tree)
set -o pipefail
out=gpurun_out/$1; shift
mkdir -p $out
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_evaluate.py tests/test_gpu_kat.py tests/test_gpu_posterior.py \
    tests/test_gpu_incremental.py -v -p no:cacheprovider --timeout 150 --timeout-method thread > $out/tests.log 2>&1
  rc=$?
  echo "tests rc=$rc: $(tail -1 $out/tests.log)"
  if [ $rc -ne 0 ]; then exit 1; fi
fi
for rep in 1 2; do
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ "$lib" = "-" ]; then unset TD_LIB_PATH; else export TD_LIB_PATH=$PWD/$lib; fi
  timeout -k 10 120 python -u tools/eval_time.py 400 > $out/$v$rep.json 2> $out/$v$rep.err
  rc=$?
  echo "$v$rep rc=$rc $(cat $out/$v$rep.json)"
  if [ $rc -ne 0 ]; then exit 1; fi
done
done
