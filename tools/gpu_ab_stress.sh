# A/B of prebuilt library variants on the stress chain (10k rays x 20k cells): stamped phases, 2000
# proposals each.  usage: tools/gpu_ab_stress.sh TAG NAME...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for v in "$@"; do
  TD_LIB_PATH=$PWD/variants/$v/libtdstar.so timeout -k 10 300 python profiles/chain_phases.py 20000 2000 10000 > $O/$v.stress.json 2>&1 || { echo "$v stress phases failed"; tail $O/$v.stress.json; exit 1; }
  python3 -c "
import json;p=json.load(open('$O/$v.stress.json'));print('$v','us/iter',round(p['us_per_iter_wall'],2),'cycles',round(p['cycles_per_iter']),{k[:8]:round(v['cycles_per_iter']) for k,v in p['phases'].items()})"
done
