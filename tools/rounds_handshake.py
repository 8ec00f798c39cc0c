#!/usr/bin/env python3
"""Diagnostic: the fixed cost of one resident tempering round (the host
handshake) against the replicas' imbalance.  Wall time per round of the
config-4 replicas for R in (1, 8) replicas and K in (1, 10) proposals per
round: with one replica there is nothing to wait for but the host; K = 1
shrinks the imbalance to one proposal's.  usage: rounds_handshake.py [rounds]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402
from bench import config4_replicas  # noqa: E402


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    out = {}
    for R in (1, 8):
        for K in (1, 10):
            chains = config4_replicas(tt, ctx, ds, 0, R)
            lad = tt.TemperingLadder(chains, tmax=8.0, seed=4242)
            lad.run(20, K)
            t0 = time.perf_counter()
            lad.run(rounds, K)
            el = time.perf_counter() - t0
            lad.close()
            t1 = time.perf_counter()
            tt.run_batch(chains, rounds * K) if R > 1 else chains[0].run(rounds * K)
            el_free = time.perf_counter() - t1
            out["R%d_K%d" % (R, K)] = {"us_per_round": round(el / rounds * 1e6, 2),
                                       "us_per_round_free_running": round(el_free / rounds * 1e6, 2)}
            print(json.dumps({"R%d_K%d" % (R, K): out["R%d_K%d" % (R, K)]}), flush=True)
            for c in chains:
                c.close()
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
