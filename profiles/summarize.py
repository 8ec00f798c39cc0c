#!/usr/bin/env python3
"""Summarise a rocprofv3 run directory (kernel_stats + per-counter PMC passes)
into a small markdown table committed under profiles/.

usage: python profiles/summarize.py gpurun_out/prof_X  > profiles/rNN_X.md
Counter conventions (MI355X_MICROARCH.md): FETCH_SIZE/WRITE_SIZE are KB per
dispatch; FETCH_SIZE under-reports wide coalesced reads by 2x on gfx950 and
is reported here both raw and doubled; SQ_WAVE_CYCLES are quad-cycles.
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    n = name.replace("tdstar::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def main(d):
    print("# rocprofv3 summary: `%s`\n" % d)
    stats = glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        print("## kernel-trace --stats\n")
        print("| kernel | calls | avg us | min us | max us | % time |")
        print("|---|---|---|---|---|---|")
        for r in csv.DictReader(open(stats[0])):
            print("| %s | %s | %.2f | %.2f | %.2f | %.2f |" % (short(r["Name"]), r["Calls"], float(r["AverageNs"]) / 1e3,
                                                          float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3,
                                                          float(r["Percentage"])))
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    if agg:
        names = sorted({c for v in agg.values() for c in v})
        print("\n## PMC counters (mean per dispatch; separate passes)\n")
        print("| kernel | " + " | ".join(names) + " | FETCH_SIZE x2 (KB) |")
        print("|---|" + "---|" * (len(names) + 1))
        for k, v in agg.items():
            if k.startswith("__amd"):
                continue
            cells = ["%.1f" % (sum(v[c]) / len(v[c])) if v.get(c) else "" for c in names]
            fx2 = "%.1f" % (2 * sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"])) if v.get("FETCH_SIZE") else ""
            print("| %s | %s | %s |" % (k, " | ".join(cells), fx2))


if __name__ == "__main__":
    main(sys.argv[1])
