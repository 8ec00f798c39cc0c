# A/B of the headline chain against ab/libtdstar_base.so, phase stamps, then the chain and evaluate parity tests
set -o pipefail
out=gpurun_out/${1:-r5b}
mkdir -p $out
TESTS=0 bash tools/gpu_ab.sh ${1:-r5b}/ab base=ab/libtdstar_base.so head= || exit 1
timeout -k 10 100 python tools/lds_plan.py > $out/lds.txt 2>&1 && cat $out/lds.txt && timeout -k 10 200 python tools/batch_phases.py 1 5000 > $out/c1.json 2>&1 || { tail $out/c1.json; exit 1; }
timeout -k 10 200 python tools/batch_phases.py 256 2000 > $out/c256.json 2>&1 || { tail $out/c256.json; exit 1; }
python -c "
import json
for f in ('c1','c256'):
    d=json.load(open('$out/'+f+'.json')); print(f, round(d['proposals_per_s']), d['total'], d['cycles_per_iter_per_chain'], 'fallbacks', d['sub_slots']['15'])
"
timeout -k 10 1200 python -u -m pytest ${TESTS_SEL:-tests/test_gpu_chain.py tests/test_gpu_bench_parity.py tests/test_gpu_incremental.py tests/test_gpu_evaluate.py} -x -q --timeout 600 --timeout-method thread > $out/tests.log 2>&1 || { echo "tests failed"; tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
