"""HBM traffic per proposal of the 256-chain launch from tools/gpu_many_traffic.sh's PMC passes:
(2 x FETCH_SIZE + WRITE_SIZE) KB (the gfx950 correction, profiles/make_traffic.py) over the dominant
k_chain_run dispatches, / (256 chains x 5000 proposals).  usage: python tools/many_traffic.py gpurun_out/OUT"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles"))
from summarize import counters, mean  # noqa: E402

KERN = "k_chain_run<true, false, 512, true, false>"
d = sys.argv[1]
for v in sorted(os.listdir(d)):
    if not os.path.isdir(os.path.join(d, v)):
        continue
    f = counters(os.path.join(d, v, "FETCH_SIZE"), True).get(KERN, {}).get("FETCH_SIZE")
    w = counters(os.path.join(d, v, "WRITE_SIZE"), True).get(KERN, {}).get("WRITE_SIZE")
    if not f or not w:
        print(v, "no counters")
        continue
    n = 256 * 5000
    print("%-10s read %.2f KB  written %.2f KB  per proposal (%d dispatches)"
          % (v, 2 * mean(f) * 1024 / n / 1024, mean(w) * 1024 / n / 1024, len(f)))
