#!/usr/bin/env python3
"""Write profiles/traffic.json (HBM bytes per launch, read by bench.py's
roofline.traffic) from the PMC passes of tools/profile.sh TAG:
traffic = FETCH_SIZE x 2 + WRITE_SIZE (KB = 1024 B), the gfx950 correction of
MI355X_MICROARCH.md, averaged over the DOMINANT dispatches of the kernel (those
lasting >= half its longest: the bench's timed launches, see summarize.py),
with the kernel trace's dominant average launch time beside it.
usage: python profiles/make_traffic.py gpurun_out/TAG TAG"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize import counters, mean, trace_rows  # noqa: E402

ROWS = {  # traffic.json key -> (run, kernel name)
    "k_chain_run/single": ("single", "k_chain_run<true, false, 512, true, false>"),
    "k_chain_run/many256": ("many", "k_chain_run<true, false, 512, true, false>"),
    "k_chain_run/many512x2": ("packed", "k_chain_run<true, false, 256, false, false>"),
    "k_nn_tile/config3": ("single", "k_nn_tile<2>"),
    "k_nn_grid/config3": ("single", "k_nn_grid"),
    "k_chain_run/stress": ("stress", "k_chain_run<false, false, 512, false, false>"),
    "k_chain_run/exchange": ("config4", "k_chain_run<true, false, 512, true, true>"),
    "k_nn_grid4/stress": ("stress", "k_nn_grid4"),
    "k_nn_tile/stress": ("stress", "k_nn_tile<2>"),
    "k_raster_brute/section": ("aux", "k_raster_brute"),
}


def main(d, tag):
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "traffic.json")
    out = {}
    if os.path.exists(path):  # rows this run has no PMC passes for keep their earlier source
        with open(path) as f:
            out = json.load(f)
    for key, (run, kern) in ROWS.items():
        agg = counters(os.path.join(d, run), True)
        v = agg.get(kern)
        if not v or not v.get("FETCH_SIZE") or not v.get("WRITE_SIZE"):
            continue
        fetch, write = mean(v["FETCH_SIZE"]), mean(v["WRITE_SIZE"])
        tr = trace_rows(os.path.join(d, run)).get(kern, [])
        dom = [x for x in tr if tr and x >= 0.5 * max(tr)]
        out[key] = {"fetch_size_kb_raw": fetch, "write_size_kb": write,
                    "traffic_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
                    "dispatches": len(v["FETCH_SIZE"]),
                    "avg_launch_us": round(mean(dom), 2) if dom else None,
                    "note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B); "
                            "KB = 1024 B; dominant dispatches (>= 1/2 the longest) only",
                    "source": "profiles/%s_%s.md" % (tag, run)}
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
