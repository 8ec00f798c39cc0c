#!/usr/bin/env python3
"""Diagnostic: where a resident tempering round's time goes (BASELINE config 4 on
one GPU: 8 replicas x 2000 cells, td_rounds_temper).  Wall time per round for
rounds of K proposals (K = 10, the bench's, and larger: the per-round overhead is
the intercept), and the replicas' stamped phase cycles (the round wait sits in
"G next proposal").  usage: rounds_phases.py [rounds]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import config4_replicas  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    out = {}
    for K in (10, 40, 160):
        chains = config4_replicas(tt, ctx, ds, 0, 8)
        lad = tt.TemperingLadder(chains, tmax=8.0, seed=4242)
        lad.run(10, K)
        L = tt.lib()
        a = [(ctypes.c_int64 * 80)() for _ in chains]
        lad.close()  # (profiling is toggled between launches)
        for c, x in zip(chains, a):
            L.tdt_chain_profile(c.h, 1, x)
        t0 = time.perf_counter()
        lad.run(rounds, K)
        el = time.perf_counter() - t0
        lad.close()
        b = [(ctypes.c_int64 * 80)() for _ in chains]
        for c, x in zip(chains, b):
            L.tdt_chain_profile(c.h, 0, x)
        per = np.array([[float(y[k] - x[k]) for k in range(14)] for x, y in zip(a, b)]) / (rounds * K)
        cyc = per.mean(axis=0)
        # each replica's own work per proposal (every stamped phase but the round wait's slot 13)
        work = per[:, [0, 1, 2, 3, 4, 5, 6, 12]].sum(axis=1)
        out[K] = {"us_per_round": round(el / rounds * 1e6, 2), "us_per_proposal_step": round(el / rounds / K * 1e6, 3),
                  "cycles_per_iter": {n: round(cyc[k], 1) for k, n in
                                      [(0, "top"), (1, "B"), (2, "C"), (3, "D"), (4, "E"), (5, "F"), (12, "G commit"),
                                       (13, "G next + round wait"), (6, "final barrier")]},
                  "work_cycles_per_iter_by_replica": [round(w, 1) for w in work],
                  "wait_cycles_per_iter_by_replica": [round(w, 1) for w in per[:, 13]]}
        for c in chains:
            c.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
