#!/usr/bin/env python3
"""Diagnostic: the config-4 replicas (8 x 2000 cells) free-running in one batch
launch, profiled: per replica the stamped cycles per proposal, the unproven grid
searches (full-scan fallbacks, prof[15]), the exact decisions (prof[65]) and the
per-action phase cycles -- what makes one replica's round of 10 proposals slow.
usage: config4_phases.py [iters]"""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402
from bench import config4_replicas  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3000
    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    chains = config4_replicas(tt, ctx, ds, 0, 8)
    temps = [8.0 ** (g / 7) for g in range(8)]
    for c, T in zip(chains, temps):
        c.set_temperature(T)
    tt.run_batch(chains, 200)
    L = tt.lib()
    a = []
    for c in chains:
        x = (ctypes.c_int64 * 80)()
        L.tdt_chain_profile(c.h, 1, x)
        a.append(np.array(x[:], dtype=np.float64))
    p0 = [np.array(c.stats()["proposed"], dtype=np.float64) for c in chains]
    acc0 = [np.array(c.stats()["accepted"], dtype=np.float64) for c in chains]
    tt.run_batch(chains, iters)
    out = []
    for c, x0, q0, c0, T in zip(chains, a, p0, acc0, temps):
        x = (ctypes.c_int64 * 80)()
        L.tdt_chain_profile(c.h, 0, x)
        d = np.array(x[:], dtype=np.float64) - x0
        st = c.stats()
        prop = np.array(st["proposed"], dtype=np.float64) - q0
        acc = np.array(st["accepted"], dtype=np.float64) - c0
        out.append({"T": round(T, 3), "ncells": st["ncells"],
                    "cycles_per_iter": round(d[[0, 1, 2, 3, 4, 5, 6, 12, 13]].sum() / iters, 1),
                    "grid_fallbacks_per_1k": round(d[15] / iters * 1e3, 2),
                    "exact_decisions_per_1k": round(d[65] / iters * 1e3, 2),
                    "accept_rate_by_action": [round(float(u / max(v, 1)), 3) for u, v in zip(acc, prop)],
                    "cycles_by_action": [round(float(d[8 + k] / max(prop[k], 1)), 1) for k in range(4)],
                    # a diagnostic build's histogram of iteration cycles (<16k, <32k, <64k, <128k, <256k, more)
                    "iter_cycles_hist": [int(d[k]) for k in (25, 35, 45, 55, 75, 79)],
                    "raw": [int(v) for v in d]})
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
