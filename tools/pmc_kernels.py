"""Mean FETCH_SIZE / WRITE_SIZE per dispatch (KB, and the gfx950 traffic FETCH x 2 + WRITE) of the
evaluate's kernels from tools/gpu_eval_traffic.sh's PMC passes.  usage: pmc_kernels.py OUT name=lib ..."""
import csv
import glob
import json
import os
import sys

out = sys.argv[1]
res = {}
for nv in sys.argv[2:]:
    v = nv.split("=", 1)[0]
    per = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        files = glob.glob(os.path.join(out, v, c, "**", "*counter_collection.csv"), recursive=True)
        acc = {}
        for f in files:
            for row in csv.DictReader(open(f)):
                if row.get("Counter_Name") != c:
                    continue
                k = row["Kernel_Name"].replace("tdstar::", "").replace("(anonymous namespace)::", "").split("(")[0]
                acc.setdefault(k, []).append(float(row["Counter_Value"]))
        for k, xs in acc.items():
            per.setdefault(k, {})[c] = round(sum(xs) / len(xs), 1)
    for k, d in per.items():
        if "FETCH_SIZE" in d and "WRITE_SIZE" in d:
            d["traffic_KB"] = round(2 * d["FETCH_SIZE"] + d["WRITE_SIZE"], 1)
    res[v] = {k: d for k, d in per.items() if k.startswith(("k_grid_fill", "k_nn_grid", "k_ray_sums"))}
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(out, "traffic.json"), "w"), indent=1)
