# HBM traffic (rocprofv3 FETCH_SIZE, WRITE_SIZE: separate passes) and speed of 256 chains per GPU for several builds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
out=gpurun_out/${1:-traffic}; shift
mkdir -p $out
A="--steps 2 --warmup 1 --no-cpu-baseline --no-full-evaluate --no-dropin --no-config4 --no-stress --batch-chains 0 --chains-per-gpu 256 --iters-per-step 5000 --no-phases"
for nv in "$@"; do
  v=${nv%%=*}; lib=${nv#*=}
  if [ -n "$lib" ]; then export TD_LIB_PATH=$PWD/$lib; else unset TD_LIB_PATH; fi
  timeout -k 10 120 python3 bench.py $A > $out/$v.json 2>&1 || { echo "$v failed"; tail -5 $out/$v.json; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/$v/fetch -o run -- python3 bench.py $A > $out/$v.fetch.log 2>&1 || { echo "$v fetch failed"; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/$v/write -o run -- python3 bench.py $A > $out/$v.write.log 2>&1 || { echo "$v write failed"; exit 1; }
  python3 - "$out" "$v" <<'PY'
import csv, json, sys, collections
out, v = sys.argv[1], sys.argv[2]
d = json.loads(open(f"{out}/{v}.json").read().strip().splitlines()[-1])
res = {}
for k in ("fetch", "write"):
    rows = [r for r in csv.DictReader(open(f"{out}/{v}/{k}/run_counter_collection.csv")) if "k_chain_run" in r["Kernel_Name"]]
    per = collections.defaultdict(float)
    for r in rows: per[r["Dispatch_Id"]] += float(r["Counter_Value"])
    vals = sorted(per.values())[-2:]
    res[k] = sum(vals) / len(vals) * 1024  # KB -> B
P = 256 * 5000
print(v, "proposals/s %.0f" % d["value"], "fetch x2 B/proposal %.0f" % (2 * res["fetch"] / P), "write B/proposal %.0f" % (res["write"] / P))
PY
done
