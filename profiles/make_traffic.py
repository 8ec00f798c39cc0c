#!/usr/bin/env python3
"""Write profiles/traffic.json (HBM bytes per launch, read by bench.py's
roofline.traffic) from the PMC passes of tools/profile.sh TAG:
traffic = FETCH_SIZE x 2 + WRITE_SIZE (KB = 1024 B), the gfx950 correction of
MI355X_MICROARCH.md.  usage: python profiles/make_traffic.py gpurun_out/TAG TAG"""
import collections
import csv
import glob
import json
import os
import sys

ROWS = {  # traffic.json key -> (run, kernel name prefix)
    "k_chain_run/single": ("single", "k_chain_run<true>"),
    "k_chain_run/many256": ("many", "k_chain_run<true>"),
    "k_nn_partial/config3": ("single", "k_nn_partial<2>"),
    "k_nn_grid/config3": ("single", "k_nn_grid"),
    "k_chain_run/stress": ("stress", "k_chain_run<false>"),
}


def short(name):
    n = name.replace("tdstar::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def counters(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(d, tag):
    out = {}
    for key, (run, kern) in ROWS.items():
        agg = counters(os.path.join(d, run))
        v = agg.get(kern)
        if not v or not v.get("FETCH_SIZE") or not v.get("WRITE_SIZE"):
            continue
        fetch = sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])
        write = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"])
        out[key] = {"fetch_size_kb_raw": fetch, "write_size_kb": write,
                    "traffic_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
                    "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B); "
                            "KB = 1024 B",
                    "source": "profiles/%s_%s.md" % (tag, run)}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
