# A/B of prebuilt library variants on one box (variants/NAME/libtdstar.so): stamped phases + the
# default single-chain bench leg, each variant twice interleaved.  usage: tools/gpu_ab.sh TAG NAME...
set -o pipefail
O=gpurun_out/$1; shift
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    TD_LIB_PATH=$PWD/variants/$v/libtdstar.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 0 --no-phases > $O/$v.$rep.bench 2>&1 || { echo "$v bench failed"; tail $O/$v.$rep.bench; exit 1; }
    python3 -c "import json;b=json.loads([l for l in open('$O/$v.$rep.bench') if l.startswith('{')][-1]);print('$v',$rep,b['value'])"
  done
done
for v in "$@"; do
  TD_LIB_PATH=$PWD/variants/$v/libtdstar.so timeout -k 10 200 python profiles/chain_phases.py 5000 20000 > $O/$v.phases.json 2>&1 || { echo "$v phases failed"; exit 1; }
  python3 -c "
import json;p=json.load(open('$O/$v.phases.json'));print('$v','cycles',round(p['cycles_per_iter']),{k[:8]:round(v['cycles_per_iter']) for k,v in p['phases'].items()})"
done
