#!/usr/bin/env python3
"""Summarise a rocprofv3 run directory (kernel trace + per-counter PMC passes)
into a small markdown table committed under profiles/.

usage: python profiles/summarize.py gpurun_out/prof_X  > profiles/rNN_X.md

A bench run launches the same kernel in several roles (a chain kernel runs
0-iteration launches at chain creation beside the timed launches), so every
table is given twice: over all dispatches, and over the DOMINANT dispatches
of each kernel -- those lasting at least half as long as its longest one,
which for the bench's timed kernels are exactly the timed launches.
bench.py's roofline numbers are checked against the dominant rows.

Counter conventions (MI355X_MICROARCH.md): FETCH_SIZE/WRITE_SIZE are KB per
dispatch; FETCH_SIZE under-reports wide coalesced reads by 2x on gfx950 and
is reported here both raw and doubled; SQ_WAVE_CYCLES are quad-cycles;
effective clock = GRBM_GUI_ACTIVE / 8 XCDs / dispatch duration.
"""
import collections
import csv
import glob
import os
import sys


def short(name):
    n = name.replace("tdstar::(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def dominant(rows, dur):
    """rows of one kernel -> the ones lasting >= half the longest."""
    if not rows:
        return rows
    top = max(dur(r) for r in rows)
    return [r for r in rows if dur(r) >= 0.5 * top]


def trace_rows(d):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            out[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return out


def counters(d, only_dominant):
    """kernel -> counter -> [values per dispatch] (and the matching durations in us)."""
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        by_k = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            by_k[(short(r["Kernel_Name"]), r["Counter_Name"])].append(r)
        for (k, c), rows in by_k.items():
            dur = lambda r: int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            sel = dominant(rows, dur) if only_dominant else rows
            per[k][c].extend(float(r["Counter_Value"]) for r in sel)
            per[k]["_us_" + c].extend(dur(r) / 1e3 for r in sel)
    return per


def mean(v):
    return sum(v) / len(v) if v else float("nan")


def table(agg):
    names = sorted({c for v in agg.values() for c in v if not c.startswith("_us_")})
    print("| kernel | dispatches | " + " | ".join(names) + " | FETCH_SIZE x2 (KB) | HBM traffic (B) | clock (GHz) |")
    print("|---|---|" + "---|" * (len(names) + 3))
    for k, v in sorted(agg.items()):
        if k.startswith("__amd"):
            continue
        cells = ["%.1f" % mean(v[c]) if v.get(c) else "" for c in names]
        fx2 = "%.1f" % (2 * mean(v["FETCH_SIZE"])) if v.get("FETCH_SIZE") else ""
        tr = "%.0f" % ((2 * mean(v["FETCH_SIZE"]) + mean(v["WRITE_SIZE"])) * 1024) \
            if v.get("FETCH_SIZE") and v.get("WRITE_SIZE") else ""
        clk = ""
        if v.get("GRBM_GUI_ACTIVE"):
            us = mean(v["_us_GRBM_GUI_ACTIVE"])
            clk = "%.2f" % (mean(v["GRBM_GUI_ACTIVE"]) / 8 / (us * 1e3)) if us > 0 else ""
        nd = max((len(x) for c, x in v.items() if not c.startswith("_us_")), default=0)
        print("| %s | %d | %s | %s | %s | %s |" % (k, nd, " | ".join(cells), fx2, tr, clk))


def main(d):
    print("# rocprofv3 summary: `%s`\n" % d)
    tr = trace_rows(d)
    if tr:
        print("## kernel trace (all dispatches, and the dominant ones: >= 1/2 the longest)\n")
        print("| kernel | calls | avg us | min us | max us | dominant calls | dominant avg us |")
        print("|---|---|---|---|---|---|---|")
        for k, v in sorted(tr.items(), key=lambda kv: -sum(kv[1])):
            dom = [x for x in v if x >= 0.5 * max(v)]
            print("| %s | %d | %.2f | %.2f | %.2f | %d | %.2f |" % (k, len(v), mean(v), min(v), max(v), len(dom),
                                                                    mean(dom)))
    for only_dom, title in ((True, "dominant dispatches"), (False, "all dispatches")):
        agg = counters(d, only_dom)
        if agg:
            print("\n## PMC counters, mean per dispatch, %s (separate passes)\n" % title)
            table(agg)


if __name__ == "__main__":
    main(sys.argv[1])
