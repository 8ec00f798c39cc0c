"""Sweep the tempering ladder's T_max at BASELINE config 4's shape (8 replicas
x 2000 cells, a swap round every 10 proposals) to find a ladder that mixes:
adjacent swap rates >= 20 % and replicas completing round trips.  One GPU,
the device-decided exchange rounds (td_rounds_exchange).

usage: python tools/calibrate_ladder.py OUT.json [rounds] [burn] [tmax ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    out = sys.argv[1]
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
    burn = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    tmaxes = [float(x) for x in sys.argv[4:]] or [1.02, 1.05, 1.1, 1.2, 1.5, 2.0, 8.0]
    import tonga

    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=4000)
    res = []
    for tmax in tmaxes:
        chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=100 + g, chain=1 + g), tt.random_model(2000, 100 + g))
                  for g in range(8)]
        lad = tt.TemperingLadder(chains, tmax=tmax, seed=4242, device_swaps=True)
        lad.run(burn, 10)
        tried0, acc0 = lad.tried.copy(), lad.accepted.copy()
        trips0 = int(lad.trips.sum())
        t0 = time.perf_counter()
        lad.run(rounds, 10)
        el = time.perf_counter() - t0
        lad.close()
        rates = [float(a) / t if t else 0.0 for a, t in zip(lad.accepted - acc0, lad.tried - tried0)]
        phis = sorted(c.stats()["phi"] for c in chains)
        r = {"tmax": tmax, "rounds": rounds, "burn": burn, "swap_rates": [round(x, 3) for x in rates],
             "min_rate": round(min(rates), 3), "round_trips": int(lad.trips.sum()) - trips0,
             "mixing": lad.mixing(), "ms_per_round": round(el / rounds * 1e3, 4),
             "phi_range": [round(phis[0], 1), round(phis[-1], 1)]}
        print(json.dumps(r), flush=True)
        res.append(r)
        for c in chains:
            c.close()
    with open(out, "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
