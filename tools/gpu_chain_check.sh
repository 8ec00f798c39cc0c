# chain kernel change: every GPU test, the stamped phases at config 3, the default bench line.  usage: TAG
set -o pipefail
O=gpurun_out/${1:-cc}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > $O/phases.json 2>&1 || { echo phases failed; tail $O/phases.json; exit 1; }
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo bench failed; tail $O/bench.log; exit 1; }
python3 -c "
import json,sys
b=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1])
print('value',b['value'],'ms/step',b['ms_per_step'],'many',b.get('many_chains',{}).get('proposals_per_s'),'stress',b.get('stress',{}).get('chain',{}).get('proposals_per_s'),'c4',b.get('config4_tempering',{}).get('ms_per_round'))
p=json.load(open('$O/phases.json')); print('cycles',p['cycles_per_iter'],{k:v['cycles_per_iter'] for k,v in p['phases'].items()}); print('Fwave',p[[k for k in p if k.startswith('F per wave')][0]])
"
[ -n "$ITEM6" ] && { TD_LDS_MODE=1 timeout -k 10 300 python tools/batch_phases.py 256 2000 > $O/batch_hbm256.json 2>&1 && timeout -k 10 300 python tools/batch_phases.py 256 2000 > $O/batch_lds256.json 2>&1 || { echo batch failed; tail $O/batch_hbm256.json; exit 1; }; }
exit 0
