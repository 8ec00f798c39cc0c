# phase stamps of one chain (and 256) for a given build (TD_LIB_PATH): outputs under gpurun_out/$1
set -o pipefail
out=gpurun_out/${1:-diag}
mkdir -p $out
[ -n "$2" ] && export TD_LIB_PATH=$PWD/$2
timeout -k 10 200 python tools/batch_phases.py 1 5000 > $out/c1.json 2>&1 || { tail $out/c1.json; exit 1; }
python -c "
import json
d=json.load(open('$out/c1.json')); print(d['total'], d['cycles_per_iter_per_chain'], d['sub_slots'])
for a,v in d['by_action'].items(): print(a, v)
"
