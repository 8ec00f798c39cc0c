"""Diagnostic: phase cycles of the device chain when C chains share one GPU
(td_chain_run_batch, one workgroup each), averaged over the chains, beside
the single-chain numbers of profiles/chain_phases.py.  usage: batch_phases.py C iters"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tonga  # noqa: E402

PHASES = ["top", "B", "C", "D", "E", "F", "G"]


def main():
    C = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    tt = tonga.load()
    ds = tt.load_data_Tonga()
    ctx = tt.TdContext.from_datastruct(ds)
    prm = tt.define_TDstructrure().replace(max_cells=10000)
    model = tt.random_model(5000, 3)
    chains = [tt.Chain(ctx, tt.chain_params(prm, ds, seed=50000 + j, chain=10000 + j), model) for j in range(C)]
    lds_mode = int(os.environ.get("TD_LDS_MODE", "0"))  # 1: the rays-in-HBM layout (testing)
    if lds_mode:
        for c in chains:
            assert tt.lib().tdt_chain_set_lds_mode(c.h, lds_mode) == 0
    tt.run_batch(chains, iters)
    L = tt.lib()
    outs0 = []
    for c in chains:
        o = (ctypes.c_int64 * 80)()
        L.tdt_chain_profile(c.h, 1, o)
        outs0.append(np.array(o[:], dtype=np.float64))
    prop0 = np.array([c.stats()["proposed"] for c in chains], dtype=np.float64).sum(0)
    t0 = time.perf_counter()
    tt.run_batch(chains, iters)
    el = time.perf_counter() - t0
    tot = np.zeros(80)
    for c, o0 in zip(chains, outs0):
        o = (ctypes.c_int64 * 80)()
        L.tdt_chain_profile(c.h, 0, o)
        tot += np.array(o[:], dtype=np.float64) - o0
    prop = np.array([c.stats()["proposed"] for c in chains], dtype=np.float64).sum(0) - prop0
    # per action (birth, death, change, move): stamped phase cycles per proposal of that action
    by_action = {}
    for a, name in enumerate(("birth", "death", "change", "move")):
        row = tot[16 + 10 * a: 16 + 10 * a + 9] / max(prop[a], 1)
        by_action[name] = {"share": round(prop[a] / max(prop.sum(), 1), 3),
                           **{p: round(x, 1) for p, x in zip(("top", "B", "C", "D", "E", "F", "G12", "G13", "G"), row)}}
    cyc = tot[:7].copy()
    cyc[6] += tot[12] + tot[13]
    n = C * iters
    print(json.dumps({"chains": C, "iters": iters, "us_per_iter_wall": el / iters * 1e6,
                      "proposals_per_s": n / el,
                      "cycles_per_iter_per_chain": {p: round(c / n, 1) for p, c in zip(PHASES, cyc)},
                      "total": round(cyc.sum() / n, 1),
                      "F per wave": [round(tot[56 + w] / n, 1) for w in range(8)],
                      # per launch, averaged over the chains: preamble (mirrors, terms, draws) and epilogue
                      "preamble cycles per launch": round(tot[76] / max(tot[78], 1), 1),
                      "epilogue cycles per launch": round(tot[77] / max(tot[78], 1), 1),
                      "launches": int(tot[78] / C), "by_action": by_action,
                      # free per-action slots (16 + 10 a + 9): sub-stamps of a diagnostic build, else 0
                      "sub_slots": {k: round(tot[k] / n, 1) for k in (11, 15, 75, 25, 35, 45, 55)},
                      # per proposal: rejected on bounds, chi^2 tail terms, exact decisions, F cycles to the
                      # scan / the decision, hit tiles, points seen, changed points, changed rays
                      "diag": {k: round(tot[k] / n, 4) for k in (14, 64, 65, 66, 67, 68, 69, 70, 71)}}, indent=1))


if __name__ == "__main__":
    main()
